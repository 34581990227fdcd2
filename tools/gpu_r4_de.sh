#!/bin/bash
set -u
bash tools/gpu_r4_d.sh || exit $?
bash tools/gpu_r4_e.sh || exit $?
