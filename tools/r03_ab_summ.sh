#!/bin/bash
# one line per bench JSON under gpurun_out/<tag>: H2D value, ms/step, in-batch acc ms, resident value, ms/step, acc ms, sync accumulate, sync reduce, parity
for f in gpurun_out/$1/*.json; do
python3 -c "import json,sys; d=json.load(open('$f')); m=d['methods']; r=m.get('ches_batch_resident',{}); print('$(basename $f .json)', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], r.get('value'), r.get('ms_per_step'), r.get('kernel_ms'), d['phases_ms']['accumulate'], d['phases_ms']['reduce'], d['parity_vs_reference'])"
done
