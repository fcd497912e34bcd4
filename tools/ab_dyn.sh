set -o pipefail
O=gpurun_out/gzpar1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gzpar_cpu.py tests/test_gzindex_cpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 600 python -u tools/fastq_rate.py > $O/fastq_rate.log 2>&1
