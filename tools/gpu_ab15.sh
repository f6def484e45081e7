set -o pipefail
mkdir -p gpurun_out
for c in 1250 10000; do for v in base db3 db4 db6 db4df8; do
if [ $v = base ]; then L=""; else L=$PWD/tools/ab/lib_$v.so; fi
LFDAS_LIB=$L timeout -k 10 200 python tools/ab_plan.py --ch $c --reps 2 "" > gpurun_out/ab_db_${v}_$c.log 2>&1 || { tail -20 gpurun_out/ab_db_${v}_$c.log; exit 1; }
echo "ch=$c $v $(grep median gpurun_out/ab_db_${v}_$c.log)"
done; done
