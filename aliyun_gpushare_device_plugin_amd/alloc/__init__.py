"""Allocation (L3 core): extender annotation protocol and the Allocate engine."""
