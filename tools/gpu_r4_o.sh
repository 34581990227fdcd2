#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r4o
MIREC_LIB=recbole_amd/_lib/alt/step_stamps.so timeout -k 10 300 python tools/probe_step_stamps.py --warmup 96 --steps 24 > gpurun_out/r4o/stamps.jsonl 2> gpurun_out/r4o/stamps.err || { tail -20 gpurun_out/r4o/stamps.err; exit 3; }
cat gpurun_out/r4o/stamps.jsonl | head -30
