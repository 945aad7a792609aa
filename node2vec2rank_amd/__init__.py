"""MI355X-native node2vec2rank fit-and-rank engine (HIP on gfx950 behind a C-ABI).

Public surface mirrors the reference package for the fit-and-rank path:
``node2vec2rank_amd.model.N2V2R`` (reference ``node2vec2rank/model.py``),
``node2vec2rank_amd.model_utils`` (reference ``node2vec2rank/model_utils.py``),
``node2vec2rank_amd.spectral.UASE`` (the ``spectral_embedding.UASE`` seam).
"""
__version__ = "0.1.0"
