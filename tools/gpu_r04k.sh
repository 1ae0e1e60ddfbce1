#!/bin/bash
# Event-timer forms: dependent-launch gap microbenchmark by event flags, the match with
# timers off / on (chained stop events vs start + stop), timer tests, a kernel trace of the
# chained form and a bench line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/r04k; mkdir -p $out
for f in 0 0x40000000 0x20000000; do timeout -k 10 60 tools/ubench_gap $f || exit 1; done > $out/ubench_flags.log 2>&1 &&
timeout -k 10 200 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "profiling or timer or async" > $out/tests.log 2>&1 &&
timeout -k 10 200 python3 tools/match_probe.py 15 > $out/match_probe_chain.log 2>&1 &&
FR_TIMER_CHAIN=0 timeout -k 10 200 python3 tools/match_probe.py 15 > $out/match_probe_startstop.log 2>&1 &&
timeout -k 10 200 python3 tools/match_probe.py 15 >> $out/match_probe_chain.log 2>&1 &&
FR_TIMER_CHAIN=0 timeout -k 10 200 python3 tools/match_probe.py 15 >> $out/match_probe_startstop.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/gap_on -o run --output-format csv -- python3 tools/gap_probe.py on 10 > $out/gap_on.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --inflight 0 --faithful-steps 0 > $out/bench.json 2> $out/bench.err &&
echo done
