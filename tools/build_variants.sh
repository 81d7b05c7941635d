#!/bin/bash
# Variant library builds for same-box bottleneck experiments (CPU side, before a GPU call):
#   bash tools/build_variants.sh NAME "-DFLAG ..." [NAME "-DFLAG ..."]...
# → mra-gan_amd/lib/var/NAME/libmragan_hip.so (objects in mra-gan_amd/build/var/NAME)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  MRAGAN_LIB_DIR=$R/mra-gan_amd/lib/var/$1 MRAGAN_OBJ_DIR=$R/mra-gan_amd/build/var/$1 MRAGAN_EXTRA_FLAGS="$2" \
    python3 "$R/mra-gan_amd/build.py" > /tmp/build_var_$1.log 2>&1 || { tail -20 /tmp/build_var_$1.log; exit 1; }
  echo "built $1"
  shift 2
done
