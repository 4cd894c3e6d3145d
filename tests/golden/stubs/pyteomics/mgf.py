"""Unused: golden capture happens at the average_spectrum() dict level."""
