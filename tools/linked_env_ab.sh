#!/bin/bash
# configs[4] linked row with and without an environment switch (ENVVAR=1), alternated
# three times: bash tools/linked_env_ab.sh ENVVAR [kinds]
V=$1
KINDS=${2:-"mixed"}
for k in $KINDS; do
  for rep in 1 2 3; do
    echo -n "base $k: "; timeout -k 10 200 python tools/linked_time.py $k 2>/dev/null || exit 1
    echo -n "$V=1 $k: "; env $V=1 timeout -k 10 200 python tools/linked_time.py $k 2>/dev/null || exit 1
  done
done
