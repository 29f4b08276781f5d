# Lone decoder window size on 128 KiB - 1 MiB blocks (after the resolve
# slice change): forced 512 / 1024 / 2048-byte windows, lone only.
set -e
cd $GRAFT_REPO_ROOT
for lw in 512 1024 2048 512 1024; do
  echo "== LZ4ADA_LONE_LW=$lw"
  for sz in 131072 262144 524288 1048576 2097152; do
    LZ4ADA_LONE_LW=$lw timeout -k 10 120 python tools/lone_time.py --size $sz --reps 50 --kinds mixed,dense,literal 2>&1 | grep -v amdgpu
  done
done
