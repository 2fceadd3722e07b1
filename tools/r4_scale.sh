cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
bash tools/shard_sweep.sh gpurun_out/r4shards > gpurun_out/r4shards_summary.txt 2>&1 || exit $?
cat gpurun_out/r4shards_summary.txt
bash tools/dist_rehearsal.sh gpurun_out/r4dist || exit $?
