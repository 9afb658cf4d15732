set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 12 "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
V=";LEOEC_GFBIT_WG=128,LEOEC_GFBIT_PF=0;LEOEC_GFBIT_LW=4,LEOEC_GFBIT_PF=0;LEOEC_GFBIT_LW=4;LEOEC_GFBIT_WG=128"
step r03_cab1 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants "$V"
step r03_cab4 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 4096 --rounds 4 --reps 6 --variants "$V"
step r03_e2e_order 600 python tools/e2e_bench.py --libs "r3:leo_erasure_amd/libleoec.so;r2:leo_erasure_amd/libleoec_r2.so" --threads 1,4 --rounds 3
echo done
