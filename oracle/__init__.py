"""ORACLE package -- test infrastructure only (see dcue_oracle.py header)."""
