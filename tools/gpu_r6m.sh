# round 6: counter passes of the secondary operations, then a cProfile of a steady LR epoch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6m}; mkdir -p $OUT
timeout -k 10 300 python -u tools/lr_he_demo.py --epochs 3 --cpu-batches 0 --sync-phases --profile-epoch 2 > $OUT/lr_prof.json 2> $OUT/lr_prof.err || { tail -n 5 $OUT/lr_prof.err; exit 3; }
bash tools/pmc_ops.sh ${1:-r6m}
