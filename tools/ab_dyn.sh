set -o pipefail
timeout -k 10 600 python -u tools/fastq_rate.py --device-gib 1 > gpurun_out/fastq_rate4.log 2>&1
