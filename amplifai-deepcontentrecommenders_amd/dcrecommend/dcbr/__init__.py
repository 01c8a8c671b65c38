"""DCBR path (BASELINE config 5): WRMF target factors + an audio ConvNet regressing them.

The reference never published `dcrecommend/dcbr` (its `.gitignore:13`), so this package restates
the papers: `wrmf.WRMF` (Hu, Koren, Volinsky 2008) and `dcbr.DCBR` (van den Oord et al. 2013).
Parity-unpinned against the reference; pinned against the oracles under oracle/.
"""
from .wrmf import WRMF, device_csr  # noqa: F401
from .dcbr import DCBR  # noqa: F401
