set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02aw
mkdir -p $OUT
timeout -k 10 120 python tools/debug/large_client.py fused > $OUT/dbg_fused.log 2>&1 || exit $?
timeout -k 10 120 python tools/debug/large_client.py fused 4000037 > $OUT/dbg_fused_small.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_large_gpu.py > $OUT/large.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/large.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/ab_frames.py tools/ab/tx_base.so tools/ab/tx_bf.so > $OUT/ab_tx.json 2> $OUT/ab_tx.err || exit $?
AB_NOCHECK=1 timeout -k 10 200 python tools/ab_frames.py tools/ab/tx_base.so tools/ab/tx_nohdr.so tools/ab/tx_bf.so > $OUT/ab_tx_diag.json 2> $OUT/ab_tx_diag.err
