"""Unused by the reference MGF path (binning.py:14 import only)."""
