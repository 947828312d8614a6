#!/bin/bash
# Ablation builds of the Welch kernel (CPU side): wc_welch.hip with one -D flag, linked with the
# product objects of every other source into tools/dbg/libwelch_<name>.so.
#   bash tools/dbg/welch_variants.sh NAME=-DFLAG ...
set -eu
cd "$(dirname "$0")/../.."
python -m nremmodfc_amd._build > /dev/null
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include $flags -c nremmodfc_amd/csrc/wc_welch.hip -o /tmp/welch_$name.o
  objs=$(ls build/product/*.o | grep -v wc_welch.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/welch_$name.o -o tools/dbg/libwelch_$name.so
  echo "built tools/dbg/libwelch_$name.so ($flags)"
done
