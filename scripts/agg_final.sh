set -o pipefail
A="--steps 1 --warmup 0 --cpu-sample 0 --no-verify"
scripts/gpu.sh bench c2agg --config c2 --agg --steps 10 --warmup 2 --cpu-sample 0 \
&& for ctr in FETCH_SIZE WRITE_SIZE; do scripts/gpu.sh pmc c2agg_$ctr $ctr --config c2 --agg $A || exit 1; done
