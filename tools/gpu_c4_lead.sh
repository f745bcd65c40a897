#!/bin/bash
# C4 (1024 pairs) with last-workgroup tails (default) vs leading-tail chains in the batched replay (NDT_BATCH_LEAD=1),
# at 2 and 3 streams.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c4lead; mkdir -p $O
for rep in 1 2; do
  for s in 3 2; do
    for lead in 0 1; do
      f=$O/c4_${rep}_s${s}_l${lead}.json
      if [ $lead = 1 ]; then export NDT_BATCH_LEAD=1; else unset NDT_BATCH_LEAD; fi
      NDT_BATCH_STREAMS=$s timeout -k 10 300 python bench.py --workload c4 --steps 1024 --no-cpu-baseline > $f 2> $f.err || { echo "c4 s$s l$lead failed"; tail -3 $f.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('rep $rep s$s lead$lead', d['value'], d.get('mean_translation_error_m'))"
    done
  done
done
