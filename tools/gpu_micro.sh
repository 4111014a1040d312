#!/bin/bash
# Microbenchmarks of memory-instruction shapes (tools/micro): one GPU call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 tools/micro/vmem 64 2000 > gpurun_out/vmem_64.jsonl 2>&1 || { cat gpurun_out/vmem_64.jsonl; exit 1; }
timeout -k 10 120 tools/micro/vmem 2048 2000 > gpurun_out/vmem_2048.jsonl 2>&1 || { cat gpurun_out/vmem_2048.jsonl; exit 1; }
cat gpurun_out/vmem_64.jsonl gpurun_out/vmem_2048.jsonl
timeout -k 10 180 tools/micro/routestore 125 1250 > gpurun_out/routestore.jsonl 2>&1 || { cat gpurun_out/routestore.jsonl; exit 1; }
cat gpurun_out/routestore.jsonl
