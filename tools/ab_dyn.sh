set -o pipefail
timeout -k 10 300 python tools/gz_par_rate.py --threads 1,8,16 > gpurun_out/gzrate3.log 2>&1 &&
timeout -k 10 600 python -u tools/fastq_rate.py --device-gib 16 > gpurun_out/fastq_rate3.log 2>&1
