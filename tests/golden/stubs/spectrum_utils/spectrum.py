"""Import-only stand-in (see the package docstring): a plain container with the
attributes benchmark.py's cosine functions and best_spectrum.py read."""


class MsmsSpectrum:
    def __init__(self, identifier=None, precursor_mz=None, precursor_charge=None, mz=None, intensity=None,
                 retention_time=None, **kw):
        self.identifier = identifier
        self.precursor_mz = precursor_mz
        self.precursor_charge = precursor_charge
        self.mz = mz
        self.intensity = intensity
        self.retention_time = retention_time
