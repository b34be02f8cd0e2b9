export F110QP_LIB=f110-mpc_amd/lib_stamps/libf110qp.so
for a in "8192 40 0 64 grouped" "8192 40 0 8 grouped" "8192 40 0 4 grouped" "65536 40 0 64 grouped" "4096 20 0 64" "4096 20 0 4" "1024 20 0 1"; do
  timeout -k 10 100 python tools/lane_stamps.py $a || exit 1
done
