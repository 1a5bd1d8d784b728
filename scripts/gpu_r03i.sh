# microbenchmarks: ILP inside the Fp2 product (tools/ilpbench), carry-chain hazard cost (tools/carrybench)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 120 ./tools/ilpbench > $O/ilpbench.json 2>&1 || exit 11
timeout -k 10 120 ./tools/carrybench > $O/carrybench.json 2>&1 || exit 12
echo done
