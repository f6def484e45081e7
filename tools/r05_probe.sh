# round-5: default bench with the sample arena
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
echo "exit $?"
