# Host-bound configs, round-2 tree (_r2tree, a git worktree of the round-2 commit) vs this tree,
# alternating on one box: papers-shaped GraphSAGE end to end.
set -o pipefail
mkdir -p gpurun_out
B="--graph papers --steps 100 --warmup 5 --no-cpu-baseline --no-traffic --no-roofline"
for T in r2 r3 r2 r3; do
  if [ $T = r2 ]; then D=_r2tree; else D=.; fi
  (cd $D && timeout -k 10 400 python bench.py $B) > gpurun_out/hostab_$T.json.tmp 2> gpurun_out/hostab_$T.err || exit 1
  tail -1 gpurun_out/hostab_$T.json.tmp >> gpurun_out/hostab_$T.json
done
echo "exit 0"
