"""numamma_amd -- MI355X-native replacement for NumaMMa's PEBS sample-analysis
loop (src/mem_sampling.c + the lookup/counter half of src/mem_analyzer.c).

The product is the C-ABI library ``libnumamma_gpu.so`` (include/numamma_gpu.h):
HIP kernels for gfx950 plus the host report writer.  This package holds the
Python handle on it (``engine``), the replay format and synthetic workload
generator (``replay``) and the multi-GPU sharding/merge driver
(``distributed``).
"""
from . import replay  # noqa: F401  (pure numpy; importable without the library)

__all__ = ["replay", "engine", "distributed"]
