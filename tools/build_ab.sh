#!/bin/bash
# Build ablib/old.so: the library with the given sources taken from git revision REV (default
# HEAD) and every other object from the current tree, for same-box A/B timing (MDG_LIB_PATH).
# usage: tools/build_ab.sh [REV] file.hip [file.hip ...]
set -eu
cd "$(dirname "$0")/.."
REV=HEAD
if git rev-parse -q --verify "$1^{commit}" > /dev/null 2>&1; then REV=$1; shift; fi
CS=mdgen_finetune_amd/csrc
make -C $CS -j8 > /dev/null
TT=$(mktemp -d)
T=$TT/x/csrc
mkdir -p $T $TT/include
cp $CS/*.hip $CS/*.h $T/
cp include/mdgen_hip.h $TT/include/
for f in "$@"; do git show "$REV:$CS/$f" > $T/$f; done
mkdir -p ablib
objs=()
for f in $CS/*.hip; do
  b=$(basename $f .hip)
  if printf '%s\n' "$@" | grep -qx "$b.hip"; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form \
      -c $T/$b.hip -o $T/$b.o
    objs+=($T/$b.o)
  else
    objs+=($CS/$b.o)
  fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "${objs[@]}" -o ablib/old.so
rm -rf $TT
echo "ablib/old.so: $* from $REV"
