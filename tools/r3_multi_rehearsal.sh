# Round 3: the driver's multi-GPU bench shapes rehearsed on one GPU: two torch.distributed ranks on device 0,
# and one process with four worker threads on device 0 (both: weak + strong points, every launch verified).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_multi}; mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --devices 0,0 > $O/bench_tr2.json 2> $O/bench_tr2.err || { tail -30 $O/bench_tr2.err; exit 1; }
cut -c1-700 $O/bench_tr2.json
timeout -k 10 400 python -u bench.py --gpus 4 --steps 5 --warmup 2 --devices 0,0,0,0 --no-cpu-baseline > $O/bench_t4.json 2> $O/bench_t4.err || { tail -30 $O/bench_t4.err; exit 1; }
python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); print(f, d['value'], d['n_gpus'], d['verified_bit_exact'], json.dumps(d.get('strong'))[:400])
" $O/bench_tr2.json $O/bench_t4.json
