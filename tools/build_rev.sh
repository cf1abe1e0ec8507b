#!/bin/bash
# tools/build_rev.sh <git-rev> <name>: build libkfec.so of an older revision into kcptube_amd/variants/<name>.so
# (A/B timing against the working tree with tools/ab.py on the same box)
set -euo pipefail
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" kcptube_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/kcptube_amd/variants"
(cd "$tmp/kcptube_amd/csrc" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result \
    -o "$root/kcptube_amd/variants/$name.so" *.hip *.cpp)
rm -rf "$tmp"
echo "$root/kcptube_amd/variants/$name.so"
