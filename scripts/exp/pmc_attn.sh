set -u
export TMPDIR=/tmp
O=gpurun_out/pmc_attn; mkdir -p $O
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
for v in 32 64; do for p in 0 4; do
  timeout -s KILL 90 rocprofv3 --pmc $C -d $O/v${v}p${p} -o pmc --output-format csv -- python scripts/attn_one.py $v $p 3 > $O/v${v}p${p}.log 2>&1 || { echo "fail $v $p"; exit 1; }
done; done
echo done
