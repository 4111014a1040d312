"""configs[3] as a whole, on the driver's GPU run: 1B records in eight
125M-record shards (bench.py's shard of rank r, 1M intervals), each analysed by
its own engine (eight ranks, all on GPU 0) in the global rank-major analysis
order, merged through numamma_amd/distributed.py's one-process-per-GPU chain
(export -> reduce / gather -> import, over gloo here, RCCL in the 8-GPU bench),
and compared counter by counter with the eight shards' bit-exact CPU
restatement merged in numpy (tools/merge8.py; the mem_sampling.c:324-342 loop
over every sample, sharded as configs[3] shards it).

Test infrastructure: the restatement (oracle/nmg_cpu_mt.cpp) is the checker.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_configs3_eight_shards_merged_bit_exact():
    # (the ranks run the restatement one at a time: 16 threads = the box's CPU
    # share; one analysis per rank)
    cmd = [sys.executable, os.path.join(ROOT, "tools", "merge8.py"), "--world", "8", "--samples", "125000000",
           "--intervals", "1000000", "--mt-threads", "16", "--reps", "1"]
    # (the ranks' progress lines on stderr, as the tool prints them)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=840)
    assert r.returncode == 0, r.stdout[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["records_total"] == 1_000_000_000
    assert out["world"] == 8 and out["intervals"] == 1_000_000
    assert out["bit_exact"], out["checks"]
    assert all(out["checks"].values())
    assert out["matched_total"] > 0 and out["page_cells"] > 0
