"""ORACLE — test infrastructure only (see kepler_oracle.h)."""
