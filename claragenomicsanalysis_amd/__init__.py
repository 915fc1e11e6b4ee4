"""MI355X-native batched POA consensus/MSA and global alignment.

Python mirror of the reference's pygenomeworks bindings (genomeworks.cudapoa,
genomeworks.cudaaligner) over the C ABI of libgwamd.so (include/*.h).  All
compute runs in hand-written HIP kernels for gfx950; there is no CPU fallback.
"""
from ._lib import load_library, library_path  # noqa: F401

__all__ = ["load_library", "library_path"]
