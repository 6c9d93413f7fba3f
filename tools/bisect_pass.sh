#!/bin/bash
# Bisect LLVM's optimisation passes for a miscompile: build one variant library
# per -opt-bisect-limit value, recompiling only the given translation unit
# (every pass numbered above the limit that can be skipped is skipped) and
# linking the product's objects for the rest.  List the numbered passes with
#   hipcc <tu_flags(tu)> <defines> --offload-device-only -c -o /dev/null <tu> -mllvm -opt-bisect-limit=-1
# Usage: tools/bisect_pass.sh <tag> <tu.hip> "<defines>" <limit>...   -> var/bisect_<tag>_<limit>.so
# (run in this container after `python __graft_entry__.py`; then, on the GPU box,
#  tools/sink_guard.py wp_crash with PAXISIM_LIB set to each variant)
set -e -o pipefail
TAG=$1; TU=$2; DEFS=$3; shift 3
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
FLAGS=$(python3 -c "import __graft_entry__ as g; print(' '.join(g.tu_flags('$TU')))")
SRCS=$(python3 -c "import __graft_entry__ as g; print(' '.join(g.HIP_SOURCES))")
SID=$(python3 -c "import __graft_entry__ as g; print(g.source_id())")
mkdir -p var build/bisect
pids=()
for L in "$@"; do
  OBJ=build/bisect/${TAG}_$L
  mkdir -p "$OBJ"
  ( /opt/rocm/bin/hipcc $FLAGS $DEFS -mllvm -opt-bisect-limit=$L -c -o "$OBJ/${TU%.hip}.o" "paxi_amd/csrc/$TU" 2> "$OBJ/bisect.log"
    printf 'extern "C" const char* paxisim_build_id(void) { return "%s"; }\n' "$SID+bisect:$TAG:$L" > "$OBJ/build_id.cpp"
    /opt/rocm/bin/hipcc -O2 -fPIC -c -o "$OBJ/build_id.o" "$OBJ/build_id.cpp"
    objs=()
    for s in $SRCS; do
      if [ "$s" == "$TU" ]; then objs+=("$OBJ/${s%.hip}.o"); else objs+=("build/hip/${s%.hip}.o"); fi
    done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "var/bisect_${TAG}_$L.so" "${objs[@]}" "$OBJ/build_id.o" -ldl ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
echo "built: $(ls var/bisect_${TAG}_*.so | tr '\n' ' ')"
