set -e
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for sm in 96 128; do
    VBFM_FORCE_SPLIT=1 VBFM_SMALL_MAX=$sm bash tools/gpu.sh ab_sm${sm}_$r bench=--rows+12500000+--steps+3+--warmup+1+--no-cpu-baseline
  done
done
