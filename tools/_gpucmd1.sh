set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 64 128 256 512 1024 2048; do
  timeout -k 10 200 python tools/gemm_bench.py --synthetic 65536 65536 $k --reps 3 > gpurun_out/g5_syn_$k.log 2>&1 || exit 1
  echo K=$k $(tail -n 2 gpurun_out/g5_syn_$k.log | awk '{print $6, $8}')
done
timeout -k 10 200 python tools/gemm_bench.py --synthetic 32768 32768 256 --reps 3 | tail -n 1
timeout -k 10 200 python tools/gemm_bench.py --synthetic 131072 131072 256 --reps 2 | tail -n 1
i=0
for c in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/g5_pmc$i -o a --output-format csv -- python3 tools/gemm_bench.py --factored --reps 2 > gpurun_out/g5_pmc$i.log 2>&1 || { echo PMCFAIL $c; tail -5 gpurun_out/g5_pmc$i.log; exit 1; }
done
echo done
