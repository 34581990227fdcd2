set -u
export TMPDIR=/tmp
O=gpurun_out/walk
mkdir -p $O
MIREC_LIB=recbole_amd/_lib/alt/walkprof.so timeout -k 10 200 python tools/probe_walk.py > $O/prof_new.log 2>&1 || { echo fail1; tail $O/prof_new.log; exit 3; }
MIREC_LIB=recbole_amd/_lib/alt/walkprof_old.so timeout -k 10 200 python tools/probe_walk.py > $O/prof_old.log 2>&1 || { echo fail2; tail $O/prof_old.log; exit 3; }
grep rep $O/prof_new.log; grep rep $O/prof_old.log
