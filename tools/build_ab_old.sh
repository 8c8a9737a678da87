#!/bin/bash
# Build the library of an earlier commit for same-box A/B runs against the
# current one (bench.py --lib build/libmastic_<tag>.so):
#   tools/build_ab_old.sh <commit> <tag>
# The old sources get the ABI-4 entry points the current binding binds
# (mastic_abi_version, mastic_set_test_hooks as a no-op,
# mastic_aggregate_device_on_stream onto the old 5-argument
# mastic_aggregate_device), so only the kernels and their host schedule differ.
# Runs on the CPU container (hipcc cross-compiles for gfx950).
set -e
COMMIT=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/build/old_$TAG
rm -rf "$D"; mkdir -p "$D/csrc" "$D/include"
for f in $(git -C "$ROOT" ls-tree --name-only "$COMMIT" draft-mouris-cfrg-mastic_amd/csrc/); do
    git -C "$ROOT" show "$COMMIT:$f" > "$D/csrc/$(basename "$f")"
done
git -C "$ROOT" show "$COMMIT:include/mastic_hip.h" > "$D/include/mastic_hip.h"
cat >> "$D/csrc/mastic_hip.hip" <<'EOF'

// ---- A/B build only (tools/build_ab_old.sh): the current binding's ABI-4 entry points
extern "C" int mastic_abi_version(void) { return 4; }
extern "C" int mastic_set_test_hooks(mastic_ctx* c, int, int) { return c ? 0 : MASTIC_EINVAL; }
extern "C" int mastic_aggregate_device_on_stream(mastic_ctx* c, int agg_id, const uint8_t* valid, void* dev,
                                                 void* stream) {
    return mastic_aggregate_device(c, agg_id, valid, dev, stream);
}
EOF
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I"$D/include" -o "$ROOT/build/libmastic_$TAG.so" \
    "$D/csrc/mastic_hip.hip"
echo "built build/libmastic_$TAG.so from $COMMIT"
