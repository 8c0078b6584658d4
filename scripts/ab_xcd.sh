set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/pv_index.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/ab_new.log 2>&1 || exit $?
SPFF_LIB=variants/libspff_noxcd.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/ab_old.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline skip > gpurun_out/ab_new2.log 2>&1 || exit $?
bash scripts/profvariants.sh variants/libspff_noxcd.so
