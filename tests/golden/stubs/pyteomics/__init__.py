"""Import-only stand-in for pyteomics (absent offline), used ONLY by
tests/golden/make_golden.py to import the reference's numeric functions.

binning.py imports ``pyteomics.mzml``/``auxiliary`` but never uses them on the
MGF path; average_spectrum_clustering.py needs ``mass.nist_mass['H+'][0][0]``.
Nothing here is product code and nothing here computes a tested result except
the proton mass constant."""
