# k_gemm_big with A fragments read two at a time ahead of their MFMAs (186 VGPRs, within the co-residency budget):
# GEMM GPU tests, then the config-2 bench against a HEAD build (_ab_head worktree), interleaved, 3 pairs
set -o pipefail
O=$PWD/gpurun_out/r05av; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # run LABEL DIR
  (cd $2 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1) || exit $?
  echo "$1 $(grep '^{' $O/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], d['parity'], r['achieved'])")"
}
for i in 1 2 3; do run new .; run head _ab_head; done
