"""Trainers of the reference (dcrecommend/nn): DCUE, over libdcue_hip."""
