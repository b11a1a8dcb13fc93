#!/bin/bash
# Strong-scaling probe on one GPU: each rank's shard of an N-way plan timed alone with S frames
# in flight (tools/shard_balance.py), plus the N=1 bench at the same S values.
export TMPDIR=/tmp
O=gpurun_out/scale
mkdir -p $O
for S in ${SP_STREAMS:-3 4}; do
  timeout -k 10 300 python tools/shard_balance.py --config c3 --worlds 2,4,8 --sides ${SP_SIDES:-32,64} --plans lpt \
    --streams $S > $O/balance_s$S.json 2> $O/balance_s$S.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/balance_s$S.json'))
print('S=$S full', d['full_frame_ms'], [(r['side'], r['world'], r['max'], r['speedup_pred']) for r in d['runs']])"
done
echo done
