#!/bin/bash
# Build a variant of libpaxisim.so with extra compile flags (A/B and diagnostics).
# Usage: tools/build_variant.sh <out.so> [-DFLAG=V ...]     (run in this container, not on the GPU box)
# BASEFLAGS replaces __graft_entry__.HIP_FLAGS (e.g. without -disable-machine-sink); the variant's build
# id is the sources' fingerprint + a hash of BASEFLAGS and the extra flags.
set -e -o pipefail
OUT=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/build/var_$(basename "$OUT" .so)
mkdir -p "$OBJ" "$(dirname "$R/$OUT")"
cd "$R"
SRCS=$(python3 -c "import __graft_entry__ as g; print(' '.join(g.HIP_SOURCES))")
tuflags() {   # the product's flags of one unit (__graft_entry__.tu_flags), or BASEFLAGS for every unit
  if [ -n "${BASEFLAGS:-}" ]; then echo "$BASEFLAGS"; else python3 -c "import __graft_entry__ as g; print(' '.join(g.tu_flags('$1')))"; fi
}
pids=()
for s in $SRCS; do
  /opt/rocm/bin/hipcc $(tuflags "$s") "$@" -c -o "$OBJ/${s%.hip}.o" "paxi_amd/csrc/$s" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
# the variant's own build id: the sources' fingerprint + its extra flags
VID="$(python3 -c "import __graft_entry__ as g; print(g.source_id())")+$(echo "${BASEFLAGS:-} $@" | md5sum | cut -c1-8)"
printf 'extern "C" const char* paxisim_build_id(void) { return "%s"; }\n' "$VID" > "$OBJ/build_id.cpp"
/opt/rocm/bin/hipcc -O2 -fPIC -c -o "$OBJ/build_id.o" "$OBJ/build_id.cpp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/$OUT" "$OBJ"/*.o -ldl
echo "built $OUT"
