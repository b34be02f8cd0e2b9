# build lib_var/<name>/libf110qp.so with the NUM = 40 solve-kernel objects (C2, C3) recompiled
# under extra -D flags (measurement only, F110QP_LIB selects it). Usage from the repo root:
# tools/build_solve_variant.sh <name> <flags...>
set -e
name=$1; shift
cd f110-mpc_amd
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc $*"
d=build_var/$name; mkdir -p $d lib_var/$name
for g in 0 1; do $H -DF110QP_NUM=40 -DF110QP_GAP=$g -c csrc/solve_inst.hip -o $d/solve_40_$g.o & done
wait
others=$(ls build_obj/*.o | grep -v "build_obj/solve_40_")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib_var/$name/libf110qp.so $others $d/*.o
echo built lib_var/$name/libf110qp.so
