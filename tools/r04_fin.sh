# Final-tree check: the full GPU suite, smoke, bench (tools/r04_full.sh),
# the lone decoder's default choice at 256 KiB - 1 MiB, the facade laps.
set -e
cd $GRAFT_REPO_ROOT
bash tools/r04_full.sh $1
for sz in 65536 131072 262144 524288 1048576; do
  timeout -k 10 120 python tools/lone_time.py --size $sz --reps 50 --kinds mixed,dense,literal 2>&1 | grep -v amdgpu
done
bash tools/r04_ftr.sh $1
