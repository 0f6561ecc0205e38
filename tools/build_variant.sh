#!/bin/bash
# Experiment build of the engine library into vlib/<name>/libpokec_fas.so (selected at run time
# with PF_LIB_PATH): a copy of the package built with extra compiler flags, e.g.
#   tools/build_variant.sh k5t K5T=1
#   tools/build_variant.sh q8 XFLAGS=-DPF_QUEUE_EXTRA=8
#   PATCH=tools/k5_exp/skip.py SKIP=terms tools/build_variant.sh noterms
#   PATCH=tools/k5_exp/k5s_slice.patch tools/build_variant.sh k5s   (then PF_DEBUG k5_slice=1)
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
mkdir -p "$tmp/pkg" "$root/vlib/$name"
cp -r "$root/recommendation-system-pokec_amd/csrc" "$root/recommendation-system-pokec_amd/Makefile" "$tmp/pkg/"
ln -s "$root/include" "$tmp/include"
# PATCH=script.py: an experiment patch run on the copied sources (python3 script.py <csrc dir>), so
# phase-skip and other throwaway experiments never live in the product kernels
# PATCH=file.patch: a git diff of the package (e.g. tools/k5_exp/k5s_slice.patch re-adds K5s, the
# wave-private slice kernel measured 20-50 % slower and kept out of the product library)
if [[ "$PATCH" == *.patch ]]; then (cd "$tmp/pkg" && patch -s -p2 < "$root/$PATCH") || { echo "patch $PATCH failed"; exit 1; }
elif [ -n "$PATCH" ]; then python3 "$PATCH" "$tmp/pkg/csrc" || { echo "patch $PATCH failed"; exit 1; }; fi
make -C "$tmp/pkg" -j8 libpokec_fas.so "$@" > "$tmp/build.log" 2>&1 || { tail -20 "$tmp/build.log"; exit 1; }
cp "$tmp/pkg/libpokec_fas.so" "$root/vlib/$name/"
rm -rf "$tmp"
echo "vlib/$name/libpokec_fas.so"
