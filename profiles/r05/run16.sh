#!/bin/bash
# round 5, call 16: the default bench line with the ResBlock kernels joined to their PMC rows
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05/pmc
timeout -k 10 900 python -u bench.py > gpurun_out/r05/pmc/bench.json 2> gpurun_out/r05/pmc/bench.err
echo "bench rc=$?"
