"""Import-only stand-in: benchmark.py imports pyteomics.parser for
fraction_of_by (out of scope); the cosine functions never touch it."""


def fast_valid(seq):
    raise NotImplementedError("pyteomics is absent offline")
