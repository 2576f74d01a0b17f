set -o pipefail
D=gpurun_out/r06b
mkdir -p $D
timeout -k 10 420 python -u tools/stress_carry.py --iters 16 --out $D/stress_carry.json > $D/stress.log 2>&1 &&
timeout -k 10 120 python -u tools/hop_latency.py --out $D/hop_latency.json > $D/hop.log 2>&1 &&
timeout -k 10 150 bash tools/acct_run.sh acct6 $D/acct6.json --steps 10 > $D/acct.log 2>&1 &&
CAIRO_ENCODE_TRACE=1 timeout -k 10 120 cairo_amd/_lib/evx1_api_caller 3840 2160 4 16 12 > $D/api.json 2> $D/api_trace.txt &&
timeout -k 10 400 python -u tools/rd_sweep.py --frames 240 --out $D/rd_sweep.json > $D/rd.log 2>&1
