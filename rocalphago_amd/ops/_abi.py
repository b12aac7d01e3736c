"""ctypes signatures of the C ABI exported by rocalphago_amd/_hipkernels.so (csrc/hip/*.hip)."""
import ctypes as C

P = C.c_void_p
I = C.c_int
F = C.c_float
I64 = C.c_int64
SZ = C.c_size_t

SIGNATURES = {
    # conv.hip
    "rag_conv_igemm": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, P, P],
    "rag_conv_igemm_cin": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, P, P, I],
    "rag_conv_wgrad_workspace": [I, I, I, I, I, P],
    "rag_conv_wgrad": [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, P, P],
    "rag_conv_wgrad_deferred": [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, P, P],
    "rag_conv_igemm_bn": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, P, P, P, P, P, P],
    "rag_conv_bn_stat_blocks": [I, I, I],
    "rag_conv_bn_fusable": [I, I, I, I, I, I],
    "rag_conv_wgrad_deferred_bn": [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, P, P, P],
    "rag_wgrad_flush": [P, P],
    "rag_wgrad_pending_bytes": [],
    "rag_wgrad_pending_init": [P],
    "rag_wgrad_pending_free": [P],
    "rag_pack_weights": [P, P, P, I, I, I, I, I, P],
    "rag_pack_trunk": [P, I, I, I64, P, I64, F, F, I],
    # conv_wino.hip (+ the pending-handle entry in conv.hip)
    "rag_conv_wino_ok": [I, I, I, I, I],
    "rag_conv_wino": [P, P, P, P, P, I, I, I, I, I, I, I, I, P],
    "rag_conv_wino_p": [P, P, P, P, P, I, I, I, I, I, I, I, I, P, P, I],
    "rag_wino_pack": [P, I, I, P, I64, F, F, I],
    "rag_pack_step": [P, I, P, I, I, I, I, P, I64, F, F, I, P, I64, I64, I64, I64],
    "rag_conv_wino_prefer": [I, I, I, I],
    "rag_conv_wino_mode": [I, I, I, I],
    "rag_conv_wino_bn_ok": [I, I, I, I],
    "rag_conv_wino_bn": [P] * 6 + [I] * 8 + [P] * 6,
    "rag_pack_input_u8": [P, P, P, P, I, I, I, I, I, I, P],
    "rag_pack_input_f32": [P, P, P, P, I, I, I, I, I, I, P],
    "rag_pack_input_bits": [P, P, P, P, I, I, I, I, I, P],
    "rag_unpack": [P, P, I, I, I, I, I, P],
    "rag_pack_nchw": [P, P, I, I, I, I, I, P],
    # head.hip
    "rag_policy_head_fwd": [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, P],
    "rag_policy_head_pass_fwd": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F,
                                 P],
    "rag_head_bwd": [P, P, P, P, P, P, P, P, I, I, I, I, I, P],
    "rag_head_bwd_m": [P, P, P, P, P, P, P, P, I, I, I, I, I, P, P, P, P, P],
    "rag_policy_head_fwd_s": [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, P],
    "rag_head_bwd_workspace": [I, I, I],
    "rag_head_linear": [P, P, P, P, I, I, I, I, P],
    "rag_value_mlp_fwd": [P, P, P, P, P, P, P, P, I, I, I, I, P],
    "rag_value_mlp_workspace": [I, I],
    "rag_value_mlp_bwd": [P] * 16 + [I, I, I, I, P],
    "rag_sl_batch": [P, P, P, I, P, I, C.c_uint, C.c_uint, P, P, I, P],
    "rag_value_batch": [P, P, P, I, C.c_uint, C.c_uint, P, P, I, P],
    "rag_value_mlp_bwd_workspace": [I, I],
    # optim.hip
    "rag_sgd": [P, P, P, I64, F, F, F, I, P],
    # rollout.hip
    "rag_rollouts": [P, P, I, I, I, F, I, P, P, C.c_uint, P, P, P, P, P, I],
    "rag_rollout_park_bytes": [I],
    # bn.hip
    "rag_bn_workspace": [I, I],
    "rag_bn_train_fwd": [P, I, I, I, I, I, P, P, P, P, F, F, P, P, P, P],
    "rag_bn_infer_coef": [P, P, P, P, F, I, P, P],
    "rag_bn_bwd_coef": [P, I, P, I, I, I, I, I, P, P, P, P, P, P, P],
    "rag_bn_apply": [P, I, P, I, P, I, P, I, P, I, I, I, I, I, P],
    "rag_bn_apply_bwd_part": [P, I, P, P, P, P, P, I, P, I, P, I, P, I, I, I, I, I, P],
    "rag_bn_finalize_fwd": [P, I, I, I, I, P, P, P, P, F, F, P, P, P],
    "rag_bn_finalize_bwd": [P, I, I, I, I, P, P, P, P, P, P],
    # sample.hip
    "rag_sample_moves": [P, P, I, P, I, I, F, C.c_uint64, P, P, P],
    # features.hip
    "rag_pass_grads": [P, P, P, P, I, I, P],
    "rag_features": [P, P, P, P, P, I, I, P, I, I, P, P, P],
    # ladder.hip
    "rag_ladder_workspace": [I, I],
    "rag_ladders": [P, P, I, I, P, P, P],
    "rag_conv_order": [I],
    "rag_conv_tap_mode": [I],
    "rag_wgrad_slab_part_bf16": [I],
    "rag_wgrad_slab_map": [I],
}

RESTYPES = {"rag_conv_wgrad_workspace": SZ, "rag_head_bwd_workspace": SZ,
            "rag_ladder_workspace": SZ, "rag_wgrad_pending_bytes": SZ,
            "rag_value_mlp_workspace": SZ, "rag_value_mlp_bwd_workspace": SZ,
            "rag_rollout_park_bytes": C.c_long}


def declare(lib):
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue  # optional kernels added in later milestones
        fn.argtypes = args
        fn.restype = RESTYPES.get(name, I)
