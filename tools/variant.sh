# Build an A/B variant of libmcaat_gpu.so with extra defines: bash tools/variant.sh <out.so> "<defines>"
# (all sources recompiled with the defines into /tmp/variant_<name>/, then linked)
set -e
OUT=$1; DEFS=$2; D=/tmp/variant_$(basename $OUT .so); mkdir -p $D
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-result"
cd "$(dirname "$0")/../mcaat_amd"
for s in alloc node_counter sdbg_build sdbg_succinct shard comm dist shard_cf cycle_finder read_mapping fastq_ingest fastq_pack instream graph_io capi; do
  /opt/rocm/bin/hipcc $F $DEFS -c csrc/$s.hip -o $D/$s.o &
done
wait
/opt/rocm/bin/hipcc $F -shared $D/*.o -o ../$OUT -lz -ldl
