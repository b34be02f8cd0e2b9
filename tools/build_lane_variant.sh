# build lib_var/<name>/libf110qp.so: the in-tree objects with the lane kernel recompiled under
# extra -D flags (measurement only: F110QP_LIB=<path> selects it in f110qp.capi)
# usage: tools/build_lane_variant.sh <name> <flags...>   (from the repo root; make -C f110-mpc_amd first)
set -e
name=$1; shift
cd f110-mpc_amd
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc $*"
d=build_var/$name; mkdir -p $d lib_var/$name
for l in 1 2 4 8 16 32 64; do $H -DF110QP_LQ=$l -c csrc/lane_inst.hip -o $d/lane_$l.o & done
$H -c csrc/lane_launch.hip -o $d/lane_launch.o &
wait
others=$(ls build_obj/*.o | grep -v -E "build_obj/lane_([0-9]+|launch)\.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib_var/$name/libf110qp.so $others $d/*.o
echo built lib_var/$name/libf110qp.so
