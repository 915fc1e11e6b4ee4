"""Loader for libgwamd.so (the HIP/gfx950 product library).

The library is built in-tree by ``python -c "import __graft_entry__ as g; g.build()"``
(or ``make -C claragenomicsanalysis_amd/csrc``).  If it is missing the import
fails loudly: there is no fallback implementation.
"""
import ctypes as C
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def library_path():
    # GWAMD_LIBRARY: an alternative in-tree build (diagnostic builds), honoured
    # only with GWAMD_DIAG=1 like the library's own tuning variables
    alt = os.environ.get("GWAMD_LIBRARY")
    if alt and os.environ.get("GWAMD_DIAG") != "1":
        sys.stderr.write("gwamd: GWAMD_LIBRARY=%s ignored without GWAMD_DIAG=1; loading the default "
                         "lib/libgwamd.so\n" % alt)
        alt = None
    return alt or os.path.join(_HERE, "lib", "libgwamd.so")


def load_library():
    global _LIB
    if _LIB is not None:
        return _LIB
    path = library_path()
    if not os.path.exists(path):
        raise ImportError(
            "libgwamd.so not built (%s); run `make -C claragenomicsanalysis_amd/csrc` or "
            "__graft_entry__.build()" % path)
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    _declare(lib)
    _LIB = lib
    return lib


def _declare(L):
    vp, i8, i16, i32, i64, sz = C.c_void_p, C.c_int8, C.c_int16, C.c_int32, C.c_int64, C.c_size_t
    P = C.POINTER
    L.gwamd_last_error.restype = C.c_char_p
    L.gwamd_last_error.argtypes = []
    L.gwamd_poa_batch_size_init.restype = i32
    L.gwamd_poa_batch_size_init.argtypes = [vp, i32, i32, i32]
    L.gwamd_poa_batch_size_init_full.restype = i32
    L.gwamd_poa_batch_size_init_full.argtypes = [vp, i32, i32, i32, i32, i32, i32]
    L.gwamd_poa_create_batch.restype = i32
    L.gwamd_poa_create_batch.argtypes = [P(vp), i32, vp, sz, i8, vp, i16, i16, i16, i32]
    L.gwamd_poa_destroy_batch.restype = None
    L.gwamd_poa_destroy_batch.argtypes = [vp]
    L.gwamd_poa_add_poa_group.restype = i32
    L.gwamd_poa_add_poa_group.argtypes = [vp, P(C.c_char_p), P(vp), P(i32), i32, P(i32)]
    for name in ("gwamd_poa_get_total_poas", "gwamd_poa_generate_poa", "gwamd_poa_batch_id",
                 "gwamd_poa_upload", "gwamd_poa_launch", "gwamd_poa_synchronize"):
        getattr(L, name).restype = i32
        getattr(L, name).argtypes = [vp]
    L.gwamd_poa_reset.restype = None
    L.gwamd_poa_reset.argtypes = [vp]
    L.gwamd_poa_get_consensus.restype = i32
    L.gwamd_poa_get_consensus.argtypes = [vp, P(i32), P(i32), P(vp), P(vp), P(i32)]
    L.gwamd_poa_get_msa.restype = i32
    L.gwamd_poa_get_msa.argtypes = [vp, P(i32), P(i32), P(vp), P(i32), P(i32)]
    L.gwamd_poa_get_graphs.restype = i32
    L.gwamd_poa_get_graphs.argtypes = [vp, P(i32), P(i32), P(vp), P(vp), P(vp), P(vp), P(i32)]
    L.gwamd_poa_get_stats.restype = i32
    L.gwamd_poa_get_stats.argtypes = [vp, P(i64), P(i32)]
    L.gwamd_poa_get_phase_ticks.restype = i32
    L.gwamd_poa_get_phase_ticks.argtypes = [vp, P(i64)]
    L.gwamd_poa_get_types.restype = i32
    L.gwamd_poa_get_types.argtypes = [vp, P(i32), P(i32)]
    L.gwamd_poa_get_capacity.restype = i32
    L.gwamd_poa_get_capacity.argtypes = [vp, P(i64), P(i32)]
    L.gwamd_poa_get_grid.restype = i32
    L.gwamd_poa_get_grid.argtypes = [vp, P(i32), P(i32)]
    L.gwamd_poa_env_tuning.restype = i32
    L.gwamd_poa_env_tuning.argtypes = [P(i32), P(i32), P(i32), P(i32)]
    L.gwamd_poa_set_spoa_accurate.restype = i32
    L.gwamd_poa_set_spoa_accurate.argtypes = [vp, i32]
    if hasattr(L, "gwamd_aligner_create"):
        from . import cudaaligner
        cudaaligner._declare(L)
    from . import cudamapper
    cudamapper._declare(L)


def last_error():
    return load_library().gwamd_last_error().decode(errors="replace")
