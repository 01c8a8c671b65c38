"""Datasets of the DCUE trainer (datasets/__init__.py:3-5 of the reference)."""
