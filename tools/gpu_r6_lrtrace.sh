# round 6: kernel trace of the LR demo (config 1) on the shipped library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r6lrtrace}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o lr --output-format csv -- \
  python3 tools/lr_he_demo.py --epochs 3 --cpu-batches 0 --sync-phases > $OUT/lr_demo.json 2> $OUT/lr_demo.err || { tail -n 5 $OUT/lr_demo.err; exit 3; }
ls $OUT/trace
