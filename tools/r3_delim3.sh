# Round 3: the newline index's shipped split (two kernels up to 512 MiB per launch, one-pass above): the whole
# GPU suite, a kernel fuzz campaign (its newline launches are all two-kernel now), the size sweep.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_delim3}; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step fuzz
timeout -k 10 150 python -u tools/fuzz_gpu.py --mode kernel --seconds 90 --seed 61 --out $O/fuzz_s61.json > $O/fuzz_s61.log 2>&1 || { tail -20 $O/fuzz_s61.log; exit 1; }
tail -n 1 $O/fuzz_s61.log | cut -c1-300
timeout -k 10 150 python -u tools/fuzz_gpu.py --mode object --seconds 60 --seed 62 --out $O/fuzz_obj_s62.json > $O/fuzz_obj_s62.log 2>&1 || { tail -20 $O/fuzz_obj_s62.log; exit 1; }
tail -n 1 $O/fuzz_obj_s62.log | cut -c1-300
step size-sweep
timeout -k 10 300 python -u tools/size_sweep.py --sizes-gib 0.0625,0.125,0.25,0.5,1,2,4,8 > $O/size_sweep.log 2>&1 || { tail -20 $O/size_sweep.log; exit 1; }
cat $O/size_sweep.log
step fastq
timeout -k 10 200 python -u tools/fastq_rate.py > $O/fastq_rate.log 2>&1 || { tail -20 $O/fastq_rate.log; exit 1; }
tail -n 6 $O/fastq_rate.log | cut -c1-300
step done
