"""DCUE model (item + user towers) on libdcue_hip."""
