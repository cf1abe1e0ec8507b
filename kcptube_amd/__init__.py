"""kcptube_amd -- MI355X-native Reed-Solomon FEC coder with kcptube's ``fec=D:R`` shard API.

The product is ``libkfec.so`` (hand-written gfx950 HIP kernels behind the C ABI in ``include/kfec.h``);
``kcptube_amd.fec.FecCode`` mirrors the reference's ``fecpp::fec_code`` over it, and
``include/fecpp_compat.hpp`` is the header-only C++ drop-in for kcptube's own sources.
"""
from .fec import FecCode, KfecError, KfecUnavailable, load_library, version  # noqa: F401

__all__ = ["FecCode", "KfecError", "KfecUnavailable", "load_library", "version"]
