# Three rocprofv3 --pmc passes (SQ group, FETCH_SIZE, WRITE_SIZE; no tracing domains) over 25 eager
# steps of the ws = 1 chain and of the forced multi-GPU chain (dist_mode 3: eager); summarise with
# scripts/pmc_summary.py.  Run through gpurun from the repo root: bash scripts/pmc_passes.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/${1:-pmc}
mkdir -p $o
B="--steps 25 --warmup 5 --no_fp32 --no_graph"
i=0
for cfg in "local|" "dist|--force_allreduce --no_placement --no_breakdown --no_chain_check --dist_mode 3"; do
  tag=${cfg%%|*}; extra=${cfg#*|}
  for pass in "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_VALU" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $o/${tag}_p$i -- python bench.py $B $extra > $o/${tag}_p$i.json 2>> $o/err.log || { echo "pass $i failed"; exit 1; }
    echo "$tag pass $i ok"
  done
done
