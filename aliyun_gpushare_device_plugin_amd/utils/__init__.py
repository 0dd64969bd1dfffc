"""Shared utilities: logging, units, metrics, stack dumps, native-library loading."""
