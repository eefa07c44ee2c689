set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02az
mkdir -p $OUT
PROBE_SET=tiles timeout -k 10 120 ./bin/hbm_probe 1024 7 > $OUT/tiles_1024MiB.json 2> $OUT/t1024.err && \
PROBE_SET=tiles timeout -k 10 120 ./bin/hbm_probe 256 9 > $OUT/tiles_256MiB.json 2> $OUT/t256.err && \
PROBE_SET=tiles timeout -k 10 120 ./bin/hbm_probe 2048 5 > $OUT/tiles_2048MiB.json 2> $OUT/t2048.err
