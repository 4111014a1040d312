"""Identity of the device code and everything that shapes its launches: a hash
of every source under numamma_amd/csrc/ (kernels, the host halves that build
partitions, size chunk pools and schedules) and of the Makefile's HIP
compiler flags.  tools/pmc_pipeline.py stamps it into
profiles/pmc_<workload>.json; bench.py reports that file's HBM traffic only
when the stamp equals the hash of the tree it runs from (counters measured on
other kernels or other launch shapes are not this launch's traffic)."""
import hashlib
import os
import re

_PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(_PKG, "csrc")
MAKEFILE = os.path.join(_PKG, "Makefile")


def kernel_sources():
    """Every file of csrc/, sorted by name."""
    return sorted(f for f in os.listdir(CSRC) if os.path.isfile(os.path.join(CSRC, f)))


def hip_flags() -> str:
    """The Makefile's HIPFLAGS line (optimisation level, arch, defines)."""
    with open(MAKEFILE) as f:
        for line in f:
            if re.match(r"\s*HIPFLAGS\s*:?=", line):
                return line.strip()
    return ""


def kernel_source_hash() -> str:
    h = hashlib.sha256()
    for name in kernel_sources():
        h.update(name.encode() + b"\0")
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(b"HIPFLAGS\0" + hip_flags().encode())
    return h.hexdigest()[:16]
