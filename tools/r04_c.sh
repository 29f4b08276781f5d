# linked row phases (sparse vs dense resolution), then the facade and the stored-copy / lead-in A/B
set -e
for d in "" 1; do
  LZ4ADA_LINKED_DENSE=$d LZ4ADA_TRACE_LINKED=1 timeout -k 10 200 python tools/linked_time.py mixed > gpurun_out/c_link$d.log 2>&1 || { tail -20 gpurun_out/c_link$d.log; exit 1; }
  grep -v Warn gpurun_out/c_link$d.log | grep -E "^\{|linked\] (init|jumps|emit|decodes|alloc|sink)" | sort | uniq -c | sort -rn | head -12
done
for lib in "" bo-lz4-ada_amd/_variants/liblz4ada_hip_lead20.so bo-lz4-ada_amd/_variants/liblz4ada_hip_lead35.so; do
  LZ4ADA_LIB=$lib timeout -k 10 150 python tools/time_decode.py --kind mixed --blocks 1024 --variant idx2 2>&1 | grep -v Warn
done
for f in "--indep 1 --block-max 4194304" "--indep 1 --block-max 65536 --blocks 256" "--indep 0 --block-max 262144 --blocks 64" "--indep 0 --block-max 65536 --blocks 256 --ccksum 0"; do
  timeout -k 10 200 python tools/facade_time.py $f --feed 4096 2>&1 | grep -v Warn
  timeout -k 10 200 python tools/facade_time.py $f --feed 0 2>&1 | grep -v Warn
done
for dec in wg lone pc; do
  LZ4ADA_FACADE_DECODER=$dec timeout -k 10 200 python tools/facade_time.py --indep 1 --block-max 65536 --raw-len 8192 --blocks 512 --feed 4096 2>&1 | grep -v Warn
done
bash tools/st_ab.sh 2>&1 | grep -v Warn | grep -E "stored"
