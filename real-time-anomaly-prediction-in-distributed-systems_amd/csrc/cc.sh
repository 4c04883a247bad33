#!/bin/bash
# cc.sh SRC OBJ FLAGS... -- compile one translation unit for gfx950 at -O3.
# LLVM's gfx950 verifier has rejected one kernel or another ("Illegal
# instruction detected: Operand has incorrect register class", a
# src_shared_base compare) at one level or another; a unit it rejects is
# rebuilt at -O2, then -O1.  The rejected level's diagnostic is printed (its
# first lines), and the level the unit finally built at is recorded in
# OBJ.lvl ("<unit> <level>"), from which the Makefile generates
# htm_build_info() -- the library reports what it was built with, and
# bench.py refuses a bench kernel not built at -O3.
set -u
src=$1
obj=$2
shift 2
log=$obj.log
for lvl in -O3 -O2 -O1; do
    if "${HIPCC:-/opt/rocm/bin/hipcc}" "$@" "$lvl" -x hip -c "$src" -o "$obj" 2>"$log"; then
        echo "$(basename "$src") $lvl" >"$obj.lvl"
        if [ "$lvl" != -O3 ]; then
            echo "  ($(basename "$src") built at $lvl)" >&2
        fi
        exit 0
    fi
    echo "  ($lvl rejected for $(basename "$src"); diagnostic:" >&2
    grep -m 8 -E "error|Illegal|LLVM ERROR" "$log" | sed 's/^/      /' >&2
    echo "  )" >&2
done
cat "$log" >&2
exit 1
