# round 4, job q: final kernels (plain nt stores again) — whole GPU suite, smoke, the driver's N=1 command, rocprofv3 evidence; then
# the A/B of `sc1 nt` through buffer stores (SML_NT_CPOL=3) vs plain nt.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04q
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 700 bash profiles/run_profiles.sh r04
rc=$?; echo "profiles rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
AB=p4app-switchml_amd/bin/ab
AB_KINDS=K1,K4,RT timeout -k 10 400 python -u tools/ab_libs_cold.py $AB/cpol0.so $AB/cpol3.so > $OUT/ab_cpol_buffer.json 2> $OUT/ab_cpol_buffer.err
echo "ab cpol buffer rc=$?"
