"""Import-only stand-in (see the package docstring): a plain container with the
two attributes benchmark.py's cosine functions read."""


class MsmsSpectrum:
    def __init__(self, identifier=None, precursor_mz=None, precursor_charge=None, mz=None, intensity=None, **kw):
        self.identifier = identifier
        self.precursor_mz = precursor_mz
        self.precursor_charge = precursor_charge
        self.mz = mz
        self.intensity = intensity
