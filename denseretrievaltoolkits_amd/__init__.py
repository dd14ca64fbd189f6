"""MI355X-native (gfx950) dense-retrieval encode-and-search hot path.

Drop-in for the bi-encoder forward, brute-force inner-product search and
in-batch score matrix of yhao-wang/DenseRetrievalToolkits (DRT).  The
arithmetic runs in hand-written HIP kernels (``csrc/``) behind the C ABI of
``include/drt.h``; Python mirrors the reference's classes.
"""
__version__ = "0.1.0"
