#!/bin/bash
# VGPR / scratch of the Fp2 leaves for a set of -D variants:  tools/micro/leaf_regs.sh "-DX=1" ...
cd "$(dirname "$0")/../.."
for v in "" "$@"; do
  d=$(mktemp -d)
  (cd $d && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $v -I "$OLDPWD/lodestar_amd/csrc" -I "$OLDPWD/include" \
     -c "$OLDPWD/tools/micro/leaf_regs.hip" -o x.o -save-temps 2>/dev/null)
  s=$(ls $d/*gfx950*.s)
  echo "== variant '$v'"
  awk '/^_Z.*:/{f=$1} /; NumVgprs:/{print f, $0} /; ScratchSize:/{print f, $0}' "$s" | grep -v "^$"
  rm -rf $d
done
