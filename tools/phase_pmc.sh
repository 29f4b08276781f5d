#!/bin/bash
# Instruction counts per decoder phase: one rocprofv3 --pmc pass (SQ_INSTS_*)
# of the decoder alone (tools/time_decode.py) for the product library and
# for every bo-lz4-ada_amd/_variants/*.so (phase-removal EXP builds: the
# difference to the product is that phase's cost).
#   bash tools/phase_pmc.sh TAG [KIND] [VARIANT]   (KIND real:NAME: bench.real_sources' blocks)
set -o pipefail
TAG=$1; KIND=${2:-mixed}; VAR=${3:-idx1}
case $KIND in real:*) KARG="--real ${KIND#real:}";; *) KARG="--kind $KIND";; esac
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/phase_${TAG}
mkdir -p $O
CTR="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
shopt -s nullglob
for lib in "" $R/bo-lz4-ada_amd/_variants/*.so; do
  name=$(basename "${lib:-product}" .so)
  (cd /tmp && export TMPDIR=/tmp && LZ4ADA_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace \
     --output-format csv -d $O/$name -o run -- python3 $R/tools/time_decode.py $KARG --variant $VAR --steps 2 \
     > $O/$name.log 2>&1) || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  grep -v amdgpu $O/$name.log | tail -1
done
# the two passes as two launches (k_index, then pass 2): per-pass counts
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace \
   --output-format csv -d $O/split -o run -- python3 $R/tools/time_decode.py $KARG --variant split --steps 2 \
   > $O/split.log 2>&1) || { echo "split failed"; tail -5 $O/split.log; exit 1; }
