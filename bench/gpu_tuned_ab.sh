set -o pipefail
mkdir -p gpurun_out/tt && cd gpurun_out/tt && \
timeout -k 10 200 python ../../bench.py --steps 20 --warmup 5 --ref-steps 0 > b_tuned.log 2>&1; tail -1 b_tuned.log | cut -c1-200; ls; \
PENROZ_TUNED_GEMMS=0 timeout -k 10 200 python ../../bench.py --steps 20 --warmup 5 --ref-steps 0 > b_default.log 2>&1; tail -1 b_default.log | cut -c1-200; \
timeout -k 10 200 python ../../bench.py --steps 20 --warmup 5 --ref-steps 0 > b_tuned2.log 2>&1; tail -1 b_tuned2.log | cut -c1-200; \
timeout -k 10 200 python ../../bench.py --model gpt2-hf --steps 10 --warmup 3 --ref-steps 0 > b_hf.log 2>&1; tail -1 b_hf.log | cut -c1-200
