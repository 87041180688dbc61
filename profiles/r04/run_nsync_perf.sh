# N = 4 (where the neighbour-wave hand-off passes the parity tests): driver bench, alternating
set -o pipefail
out=gpurun_out/r04/nsync; mkdir -p $out
bash profiles/r04/ab_libs.sh $out adjoint-ode-adaptivity_amd/lib/ab/libdgadv_base.so adjoint-ode-adaptivity_amd/lib/ab/libdgadv_nsync.so || exit 1
echo all-done
