# Lone decoder on small blocks: forced 512 / 1024-byte windows (lone only).
set -e
cd $GRAFT_REPO_ROOT
for lw in 512 1024 512 1024; do
  echo "== LZ4ADA_LONE_LW=$lw"
  for sz in 16384 32768 65536 131072; do
    LZ4ADA_LONE_LW=$lw timeout -k 10 120 python tools/lone_time.py --size $sz --reps 50 --kinds mixed,dense,literal 2>&1 | grep -v amdgpu
  done
done
