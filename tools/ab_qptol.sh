cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/ab_qptol; mkdir -p $O
for cfg in "1e-8 1024" "1e-6 1024" "1e-8 128" "1e-6 128" "1e-7 1024"; do
  set -- $cfg
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --qp-tol $1 --batch $2 --no-cpu-baseline > $O/b_$1_$2.json 2> $O/b_$1_$2.err || exit $?
done
