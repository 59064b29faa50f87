set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tile2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in t32x8 t16x16; do
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$v.so timeout -k 10 300 python tools/ab_time.py --scenes 6 8 3 1 --modes 1 --tag $v >> $O/ab.jsonl 2>> $O/err || exit 1
  MCPT_LIB=montecarlo-pathtracing_amd/mcpt/variants/libmcpt_$v.so timeout -k 10 300 python tools/shard_balance.py --bands 8 > $O/bal_$v.jsonl 2>> $O/err || exit 1
done
python -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['scene'], d['msamples_s'])
for v in ['t32x8','t16x16']:
    for l in open('$O/bal_'+v+'.jsonl'):
        d=json.loads(l); print(v, d['case'], d['slowest_ms'], d['balance'], d['projected_msamples_s'])"
