# K1 access-shape A/B: loads-only stream of K1's shape
# (16 rows x 64 B per wave instruction) vs whole 128-B lines (8 rows x 128 B),
# full width and the 8-GPU shard width, own allocation.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for nch in 10000 1248; do
  for shape in 0 1 0 1; do
    timeout -k 5 60 tools/ubench_narrow $nch $nch 0 32 0 $shape || exit $?
  done
done
