#!/bin/bash
# A/B of engine builds under variants/*.so: correctness probe, bench value,
# and the HBM write traffic of the whole isolated chain (PMC WRITE_SIZE).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/ab
for so in variants/*.so; do
  n=$(basename $so .so)
  echo "== $n"
  TBG_LIB=$R/$so timeout -k 10 120 python -u tools/probe_small.py > gpurun_out/ab/$n.probe 2>&1 || { echo "probe failed"; tail -3 gpurun_out/ab/$n.probe; exit 1; }
  tail -2 gpurun_out/ab/$n.probe | head -1
  TBG_LIB=$R/$so timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { tail -3 gpurun_out/ab/$n.err; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/ab/$n.json
  (cd /tmp && TBG_LIB=$R/$so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/ab/pmc_$n -o run -- python3 $R/bench.py --no-cpu --steps 2 --inflight 1 > $R/gpurun_out/ab/pmc_$n.log 2>&1) || echo "pmc failed"
done
