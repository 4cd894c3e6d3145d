"""Import-only stand-in for spectrum_utils (absent offline), used ONLY by
tests/golden/make_golden.py so the reference's benchmark.py can be imported.
cos_dist/average_cos_dist (benchmark.py:19-38) only read ``.mz`` and
``.intensity``; nothing here computes a tested value."""
