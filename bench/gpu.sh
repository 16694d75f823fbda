# GPU-box driver: one parameterised script for every recurring GPU step (run via gpurun).
#
#   bash bench/gpu.sh check                  GPU tests + smoke + headline bench
#   bash bench/gpu.sh tests [-k EXPR]        GPU tests only (optionally a subset)
#   bash bench/gpu.sh bench [bench.py args]  headline bench (default 20 timed / 5 warmup steps)
#   bash bench/gpu.sh ab "VAR=a" "VAR=b"     same-box A/B of the headline bench, two passes
#                                            (any arms x workloads: python bench/ab.py --help)
#   bash bench/gpu.sh prof [tag] [-- cmd]    rocprofv3 kernel trace + per-step summary (default cmd:
#                                            the headline bench, 3 warmup + 5 timed steps)
#   bash bench/gpu.sh pmc tag KERNELS -- cmd  the standard PMC passes (timing/LDS, instruction mix,
#                                            HBM fetch, HBM write) over cmd, summed per kernel whose
#                                            name contains one of the comma-separated KERNELS
#   bash bench/gpu.sh decode [gpt2|gemma3-1b] decode bench: eager, graph; batch 64 and 1
#   bash bench/gpu.sh gemma-train            Gemma-3 1B shaped training bench, B = 8 and 16
#   bash bench/gpu.sh gemma4-train           Gemma-4-class (gemma4-e2b config) training bench, B = 8
#   bash bench/gpu.sh attn                   flash attention vs SDPA, head_dim 64 / 128 / 256
#   bash bench/gpu.sh ddp                    2-rank data-parallel rehearsal on one GPU (gloo)
#
# Every GPU step runs under its own timeout and a failing step ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cmd=${1:-check}
shift || true

tests() {
  timeout -k 10 500 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 120 --timeout-method thread "$@" \
    > gpurun_out/pytest_gpu.log 2>&1; local rc=$?
  grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
  tail -3 gpurun_out/pytest_gpu.log
  return $rc
}

bench() {
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/bench.log 2>&1 \
    || { tail -20 gpurun_out/bench.log; return 1; }
  grep '^{' gpurun_out/bench.log
}

case $cmd in
  check)
    tests || exit 1
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
      || { tail -20 gpurun_out/smoke.log; exit 1; }
    tail -1 gpurun_out/smoke.log
    bench --ref-steps 0 ;;
  tests) tests "$@" ;;
  bench) bench "$@" ;;
  ab)
    args=(); i=0
    for e in "$@"; do args+=(--arm "arm$i:$e"); i=$((i+1)); done
    timeout -k 10 1000 python bench/ab.py "${args[@]}" --work headline --log gpurun_out/ab.jsonl || exit 1 ;;
  prof)
    tag=${1:-prof}; shift || true
    steps=8
    if [ "$1" = "--" ]; then shift; else set -- python3 bench.py --steps 5 --warmup 3 --ref-steps 0; fi
    [ -n "$PROF_STEPS" ] && steps=$PROF_STEPS
    timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/$tag -o run -- "$@" > gpurun_out/$tag.log 2>&1 \
      || { tail -20 gpurun_out/$tag.log; exit 1; }
    DB=$(find gpurun_out/$tag -name 'run_results.db' | head -n1)
    python3 bench/prof_summary.py $DB --steps $steps --top ${PROF_TOP:-30} $PROF_ARGS > gpurun_out/${tag}_summary.txt || exit 1
    rm -rf gpurun_out/$tag
    head -n ${PROF_TOP:-40} gpurun_out/${tag}_summary.txt | cut -c1-160 ;;
  pmc)
    tag=$1; kernels=$2; shift 2; [ "$1" = "--" ] && shift
    mkdir -p gpurun_out/pmc_$tag
    pass() {
      timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmc_$tag/$2 -o p -- "${@:3}" \
        > gpurun_out/pmc_$tag/$2.log 2>&1 || { tail -5 gpurun_out/pmc_$tag/$2.log; return 1; }
    }
    pass "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" a "$@" && \
    pass "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" b "$@" && \
    pass "FETCH_SIZE" c "$@" && pass "WRITE_SIZE" d "$@" || exit 1
    python3 bench/pmc_summary.py gpurun_out/pmc_$tag "$kernels" | tee gpurun_out/pmc_${tag}_summary.txt ;;
  decode)
    model=${1:-gpt2}
    for e in "PENROZ_GRAPH_DECODE=0" "PENROZ_GRAPH_DECODE=1"; do
      for b in 64 1; do
        env $e timeout -k 10 240 python bench/bench_decode.py --model $model --batch $b > gpurun_out/dec.log 2>&1 \
          || { tail -20 gpurun_out/dec.log; exit 1; }
        echo "$e B$b $(grep metric gpurun_out/dec.log)"
      done
    done ;;
  decode-ab)
    # same-box A/B of an env switch on the graph decode program, two interleaved passes
    model=$1; var=$2; shift 2
    for pass in 1 2; do
      for b in "$@"; do
        for v in 0 1; do
          env PENROZ_GRAPH_DECODE=1 $var=$v timeout -k 10 240 python bench/bench_decode.py --model $model --batch $b \
            > gpurun_out/dec.log 2>&1 || { tail -20 gpurun_out/dec.log; exit 1; }
          echo "pass$pass $var=$v B$b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dec.log)"
        done
      done
    done ;;
  gemma-train)
    for B in 8 16; do
      timeout -k 10 400 python bench.py --model gemma3-1b --batch $B --steps 5 --warmup 2 --ref-steps 0 \
        > gpurun_out/gemma_train_b$B.log 2>&1 || { tail -30 gpurun_out/gemma_train_b$B.log; exit 1; }
      grep '^{' gpurun_out/gemma_train_b$B.log | cut -c1-400
    done ;;
  gemma4-train)
    timeout -k 10 400 python bench.py --model gemma4-e2b --batch 8 --steps 5 --warmup 2 --ref-steps 0 \
      > gpurun_out/gemma4_train_b8.log 2>&1 || { tail -30 gpurun_out/gemma4_train_b8.log; exit 1; }
    grep '^{' gpurun_out/gemma4_train_b8.log | cut -c1-400 ;;
  attn)
    for cfg in "--B 64 --T 1024 --H 12 --Hkv 12 --D 64" "--B 16 --T 2048 --H 16 --Hkv 8 --D 128" \
               "--B 16 --T 2048 --H 4 --Hkv 1 --D 256" "--B 8 --T 4096 --H 4 --Hkv 1 --D 256" \
               "--B 8 --T 1024 --H 8 --Hkv 1 --D 512" "--B 8 --T 1024 --H 8 --Hkv 1 --D 256"; do
      timeout -k 10 120 python bench/attn_bench.py $cfg --iters 10 --sdpa > gpurun_out/attn.log 2>&1 \
        || { tail -20 gpurun_out/attn.log; exit 1; }
      grep '^{' gpurun_out/attn.log | tee -a gpurun_out/attn_all.jsonl
    done ;;
  ddp)
    export PENROZ_BENCH_DEVICE=0 PENROZ_DIST_BACKEND=gloo
    timeout -k 10 240 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 200 --timeout-method thread \
      > gpurun_out/ddp_test.log 2>&1 || { tail -40 gpurun_out/ddp_test.log; exit 1; }
    tail -3 gpurun_out/ddp_test.log
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 16 > gpurun_out/ddp_bench.log 2>&1 \
      || { tail -40 gpurun_out/ddp_bench.log; exit 1; }
    grep metric gpurun_out/ddp_bench.log ;;
  *) echo "unknown step: $cmd"; exit 2 ;;
esac
