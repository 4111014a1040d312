"""Identity of the device code: a hash of the HIP sources and headers the
attribution kernels are built from.  tools/pmc_pipeline.py stamps it into
profiles/pmc_<workload>.json; bench.py reports that file's HBM traffic only
when the stamp equals the hash of the tree it runs from (counters measured on
other kernels are not this kernel's traffic)."""
import hashlib
import os

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
KERNEL_SOURCES = ("nmg_device.h", "nmg_engine.hip", "nmg_internal.h", "nmg_kernels.h", "nmg_kernels.hip",
                  "nmg_route.h", "nmg_route.hip")


def kernel_source_hash() -> str:
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        h.update(name.encode() + b"\0")
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
