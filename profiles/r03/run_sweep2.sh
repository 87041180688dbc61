# Dataflow sweep variants: occupancy (natural 88 VGPRs = 2 workgroups/CU vs forced 6 waves/SIMD,
# 80 VGPRs + spills = 3/CU), sc1 loads vs plain loads (timing only), 20- vs 10-step forward
# blocks, against the launch chains (DG_REC_SWEEP=0).
bash profiles/r03/ab_sweep.sh gpurun_out/r03/sweep2 lc=DG_REC_SWEEP=0 base=- w6=DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/exp/libdgadv_w6.so w6plain=DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/exp/libdgadv_w6plain.so w6f10=DG_LIB_PATH=adjoint-ode-adaptivity_amd/lib/exp/libdgadv_w6.so,DG_REC_FWD_STEPS_PER_LAUNCH=10
