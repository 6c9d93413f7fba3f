#!/bin/bash
# Build a variant of libpaxisim.so that recompiles only some translation units
# with extra flags and links the default build's objects for the rest (A/B of
# one kernel instance without a full rebuild).  Run `python __graft_entry__.py` first.
# Usage: tools/build_variant_tu.sh <out.so> "<k_x.hip k_y.hip>" [-DFLAG=V ...]
# (BASEFLAGS replaces __graft_entry__.HIP_FLAGS for those units, as in build_variant.sh)
set -e -o pipefail
OUT=$1; TUS=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/build/var_$(basename "$OUT" .so)
mkdir -p "$OBJ" "$(dirname "$R/$OUT")"
cd "$R"
tuflags() {   # the product's flags of one unit (__graft_entry__.tu_flags), or BASEFLAGS for every unit
  if [ -n "${BASEFLAGS:-}" ]; then echo "$BASEFLAGS"; else python3 -c "import __graft_entry__ as g; print(' '.join(g.tu_flags('$1')))"; fi
}
SRCS=$(python3 -c "import __graft_entry__ as g; print(' '.join(g.HIP_SOURCES))")
objs=()
pids=()
for s in $SRCS; do
  if [[ " $TUS " == *" $s "* ]]; then
    /opt/rocm/bin/hipcc $(tuflags "$s") "$@" -c -o "$OBJ/${s%.hip}.o" "paxi_amd/csrc/$s" &
    pids+=($!)
    objs+=("$OBJ/${s%.hip}.o")
  else
    objs+=("build/hip/${s%.hip}.o")
  fi
done
for p in "${pids[@]}"; do wait "$p"; done
# the variant's own build id: the sources' fingerprint + its extra flags
VID="$(python3 -c "import __graft_entry__ as g; print(g.source_id())")+$(echo "${BASEFLAGS:-} $TUS $@" | md5sum | cut -c1-8)"
printf 'extern "C" const char* paxisim_build_id(void) { return "%s"; }\n' "$VID" > "$OBJ/build_id.cpp"
/opt/rocm/bin/hipcc -O2 -fPIC -c -o "$OBJ/build_id.o" "$OBJ/build_id.cpp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/$OUT" "${objs[@]}" "$OBJ/build_id.o" -ldl
echo "built $OUT"
