#!/bin/bash
# Round-2 baseline pass on the GPU box: the VALU rate sweep (1/2/4/8 waves per
# SIMD), the bench at HIP's default 4 hardware queues and at 16, and a
# rocprofv3 kernel-trace of one batch in flight (exclusive kernel times).
# Every GPU step is bounded; the script stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02_base
mkdir -p $O
cd $R
echo "host: nproc=$(nproc) cpu_count=$(python3 -c 'import os;print(os.cpu_count(), len(os.sched_getaffinity(0)))')" | tee $O/host.txt
echo "== valu_rates"; timeout -k 10 120 tools/microbench/valu_rates 2000 > $O/valu_rates.txt 2>&1; cat $O/valu_rates.txt
echo "== bench q4"; timeout -k 10 200 python bench.py --no-cpu --hw-queues 4 > $O/bench_q4.json 2> $O/bench_q4.err || { tail -5 $O/bench_q4.err; exit 1; }
cut -c1-200 $O/bench_q4.json
echo "== bench q16"; timeout -k 10 200 python bench.py --no-cpu --hw-queues 16 > $O/bench_q16.json 2> $O/bench_q16.err || { tail -5 $O/bench_q16.err; exit 1; }
cut -c1-200 $O/bench_q16.json
cd /tmp
export TMPDIR=/tmp
echo "== rocprof inflight 1"; timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_iso -o run -- python3 $R/bench.py --no-cpu --inflight 1 --steps 6 --warmup 1 > $O/prof_iso.json 2> $O/prof_iso.log || { tail -20 $O/prof_iso.log; exit 1; }
echo "== done"
