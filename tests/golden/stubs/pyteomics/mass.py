"""Only the constant average_spectrum_clustering.py:6 reads (proton mass, NIST)."""
nist_mass = {'H+': {0: (1.00727646677, 1.0)}}
