#!/bin/bash
# Build the library of an earlier commit for same-box A/B runs against the
# current one (bench.py --lib build/libmastic_<tag>.so):
#   tools/build_ab_old.sh <commit> <tag>
# The current binding (mastic_amd/_lib.py) checks mastic_abi_version() and
# binds every entry point of the current header, so the old sources get:
#   * mastic_abi_version() returning the current ABI (the old definition, if
#     any, is renamed away);
#   * mastic_aggregate_device_on_stream forwarding to the old 5-argument
#     mastic_aggregate_device when the old source lacks it (rounds <= 3);
#   * a stub returning MASTIC_ENODEV for every other entry point the old
#     source does not define (e.g. the round-5/6 communicator calls), which
#     the A/B benches never call.
# So only the kernels and their host schedule differ.  RCCL is dlopened by
# ABI-6 sources; older ones link it (-lrccl below).  Runs on the CPU
# container (hipcc cross-compiles for gfx950).
set -e
COMMIT=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/build/old_$TAG
rm -rf "$D"; mkdir -p "$D/csrc" "$D/include"
for f in $(git -C "$ROOT" ls-tree --name-only "$COMMIT" draft-mouris-cfrg-mastic_amd/csrc/); do
    git -C "$ROOT" show "$COMMIT:$f" > "$D/csrc/$(basename "$f")"
done
git -C "$ROOT" show "$COMMIT:include/mastic_hip.h" > "$D/include/mastic_hip.h"
python3 - "$ROOT" "$D" <<'EOF'
import re, sys
root, d = sys.argv[1], sys.argv[2]
sys.path.insert(0, root + "/draft-mouris-cfrg-mastic_amd")
from mastic_amd import _lib
src_path = d + "/csrc/mastic_hip.hip"
src = open(src_path).read()
defined = set(re.findall(r'extern "C"[^(]*?\b(mastic_[a-z_0-9]+)\s*\(', src))
app = ["", "// ---- A/B build only (tools/build_ab_old.sh): the current binding's entry points",
       "#undef mastic_abi_version",
       'extern "C" int mastic_abi_version(void) { return %d; }' % _lib.ABI_VERSION]
for name in _lib.EXPORTS:
    if name in defined or name == "mastic_abi_version":
        continue
    if name == "mastic_aggregate_device_on_stream" and "mastic_aggregate_device" in defined:
        app.append('extern "C" int mastic_aggregate_device_on_stream(mastic_ctx* c, int agg_id, const uint8_t* valid, '
                   'void* dev, void* stream) { return mastic_aggregate_device(c, agg_id, valid, dev, stream); }')
    else:
        app.append('extern "C" int %s(...) { return MASTIC_ENODEV; }' % name)
# the old definition of mastic_abi_version (if any) is renamed by a macro that
# the appendix #undefs before its own
open(src_path, "w").write("#define mastic_abi_version mastic_abi_version_old\n" + src + "\n".join(app) + "\n")
EOF
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I"$D/include" -o "$ROOT/build/libmastic_$TAG.so" \
    "$D/csrc/mastic_hip.hip" -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl
echo "built build/libmastic_$TAG.so from $COMMIT"
