#!/bin/bash
# Build a variant of the HIP library for tools/ab.py:
#   tools/mkvariant.sh NAME PATCH   (PATCH: python file or snippet editing `src`,
#                                    a dict filename -> text of doorman_amd/csrc)
set -eu
NAME=$1; PATCH=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/variant_$NAME
rm -rf $W; mkdir -p $W/x/csrc $W/include
cp $ROOT/doorman_amd/csrc/*.hip $ROOT/doorman_amd/csrc/*.cpp $ROOT/doorman_amd/csrc/*.h $ROOT/doorman_amd/csrc/Makefile $W/x/csrc/
cp $ROOT/include/doorman_hip.h $W/include/
python3 - "$W/x/csrc" "$PATCH" <<'PY'
import glob, os, sys
d, patch = sys.argv[1], sys.argv[2]
src = {os.path.basename(f): open(f).read() for f in glob.glob(d + "/*")}
code = open(patch).read() if os.path.exists(patch) else patch
exec(code)
for k, v in src.items():
    open(os.path.join(d, k), "w").write(v)
PY
mkdir -p $ROOT/tools/variants
make -s -C $W/x/csrc OUT=$ROOT/tools/variants/lib_$NAME.so >/dev/null
echo $ROOT/tools/variants/lib_$NAME.so
