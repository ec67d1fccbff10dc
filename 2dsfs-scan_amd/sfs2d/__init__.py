"""sfs2d: MI355X-native windowed 2D-SFS composite-likelihood scan (host side).

Layers: ``pack`` (SNP dict -> SoA), ``_lib`` (ctypes over include/sfs2d.h), ``engine``
(contexts, resident data, plans), ``post`` (the reference drivers' sequential semantics),
``vcf`` (native VCF + popmap ingest), ``synth`` (seeded synthetic streams), ``dist`` (one process per GPU).
"""
from .pack import PackedSNPs, pack_snp_dict, to_snp_dict  # noqa: F401

__version__ = "0.1.0"
