"""charon_amd: MI355X-native threshold-BLS engine for Charon's signature hot path.

``charon_amd.tbls`` mirrors the reference Go package ``tbls`` (tbls/tss.go);
``charon_amd.engine`` is the ctypes handle on libtbls_gpu.so (include/tbls_gpu.h).
"""
__all__ = ["engine", "tbls"]
