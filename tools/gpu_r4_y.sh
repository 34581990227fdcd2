#!/bin/bash
# Round-4: the driver window's kernel timeline (first model step after t0, waits).
set -u
export TMPDIR=/tmp
bash tools/trace_short.sh || exit 5
cat gpurun_out/prof_short/tw.txt | head -80
