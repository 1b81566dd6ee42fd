#!/bin/bash
# Sweep of the bench's launch shape: batches per launch (--merge) x launches
# in flight (--inflight), "m:i" pairs in MERGE_SWEEP, hardware queues in Q_SWEEP.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/merge
mkdir -p $O
cd $R
for q in ${Q_SWEEP:-4 16}; do
for mi in ${MERGE_SWEEP:-1:8 4:2 4:4 8:1 8:2 12:2}; do
  m=${mi%:*}; i=${mi#*:}
  st=$((m * 3)); [ $st -lt 24 ] && st=$(( (24 / m) * m ))
  timeout -k 10 300 python bench.py --no-cpu --api-batches 0 --hw-queues $q --merge $m --inflight $i --steps $st --warmup $m > $O/q${q}_m${m}_i${i}.json 2> $O/q${q}_m${m}_i${i}.err || { echo "fail q$q m$m i$i"; tail -3 $O/q${q}_m${m}_i${i}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/q${q}_m${m}_i${i}.json'));print('q$q m$m i$i', d['value'], d['ms_per_step'])"
done; done
