set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
A="--model EA_GNN --bf16 --config cfg5 --steps 6 --warmup 2 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 300 python bench.py $A > gpurun_out/abea_on_$i.json 2>/dev/null || exit 3
  timeout -k 10 300 python bench.py $A --py-set bgnn.ea.RESIDUAL_EPILOGUE=False > gpurun_out/abea_off_$i.json 2>/dev/null || exit 3
done
