set -o pipefail
out=gpurun_out/r04b; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "export_async" > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -2 $out/t.log
timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > $out/b2.json 2> $out/b2.err || { tail -30 $out/b2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/b2.json'))
print('n_gpus', d['n_gpus'], 'shard', d['config']['shard'], 'ms=%.3f value=%.0f' % (d['ms_per_step'], d['value']), d['result_decrypted'], d['result_expected'], d['results_ok_steps'])
print('per_rank', d['per_rank']); print('lat', d['step_latency']); print('weak_matches', d['weak_matches'])"
