#!/bin/bash
# Ablation builds of one source (CPU side): csrc/<SRC>.hip with extra -D flags, linked with the
# product objects of every other source into tools/dbg/lib<SRC>_<name>.so.
#   bash tools/dbg/variants.sh SRC NAME=-DFLAG ...      (e.g. wc_sde half=-DWC_ZMEM_HALF=1)
set -eu
cd "$(dirname "$0")/../.."
SRC=$1; shift
python -m nremmodfc_amd._build > /dev/null
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include $flags -c nremmodfc_amd/csrc/$SRC.hip -o /tmp/${SRC}_$name.o
  objs=$(ls build/product/*.o | grep -v "/$SRC.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/${SRC}_$name.o -o tools/dbg/lib${SRC}_$name.so
  echo "built tools/dbg/lib${SRC}_$name.so ($flags)"
done
