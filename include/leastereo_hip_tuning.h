/*
 * leastereo_hip_tuning.h -- tuning hooks of libleastereo_hip.so (not part of the
 * drop-in contract in leastereo_hip.h).
 *
 * Each hook overrides a planner choice of one engine for A/B measurements and the
 * sweep tools under tools/ (conv_sweep.py, wino_sweep.py, wino2_sweep.py,
 * resample_probe.py, gpu_ab.sh via the LEASTEREO_* variables of _lib.py).  The
 * settings are process-wide (every host thread sees them) and take effect on the
 * next launch; callers of the hot path never need them.  Each returns 0, or
 * LEA_E_INVALID for an out-of-range value (nothing changed).
 */
#ifndef LEASTEREO_HIP_TUNING_H
#define LEASTEREO_HIP_TUNING_H

#ifdef __cplusplus
extern "C" {
#endif

/* Direct k = 3 engine: force the (NT, TW, TD) tile (nt <= 0 restores the planner).
 * A tile not instantiated for the conv's cout block makes the conv return
 * LEA_E_UNSUPPORTED (tools/conv_sweep.py). */
int lea_conv3d_set_tile_override(int nt, int tw, int td);

/* 1 (default) = lea_conv3d_bnrelu_resampled with k = 1 and at most 131072 output
 * voxels (B x D x H x W) on the gather-GEMM (each lane interpolates its own MFMA
 * operand from the 8 corners, no staging), 0 = always the register-staged engine. */
int lea_conv3d_set_rs_gather(int on);

/* 1 (default) = the fp32 1x1 streaming kernel ("conv1x1_kernel") gives each lane NT
 * consecutive voxels, so its loads, residual reads and stores are NT-float vectors (when
 * every base, batch stride and D*H*W is a multiple of NT floats), 0 = one float per lane
 * and tile.  Bit-identical. */
int lea_conv1x1_set_vector(int on);

/* bf16 engine: force the conv tile -- th rows, td planes, mt 16-row tiles per wave
 * (th <= 0 restores the planner; tools/conv_sweep.py --bf16). */
int lea_conv3d_bf16_set_tile_override(int th, int td, int mt);

/* bf16 engine variant: 0 = the planner's choice (single-chunk 3x3x3 layers, cin <= 16,
 * stream along D: "conv_bf16_stream_kernel<MT, WC, TH, NB>"), 1 = the tile kernel for
 * every layer. */
int lea_conv3d_bf16_set_variant(int variant);

/* 1 (default) = lea_conv3d_bnrelu_bf16 with k = 1 and cin <= 128 on the streamed 1x1
 * kernel (each lane loads its own 16-byte B word, weights in registers, no staging;
 * bit-identical to the tile kernel), 0 = the tile kernel. */
int lea_conv3d_bf16_set_stream1x1(int on);

/* LEA_PAIR_SUM on the bf16 engine: 3 (default) = the 8 -> 8 steps (cout <= 8) on the split-wave
 * pair kernel's plane-paired tile ("conv_bf16_pair_kernel<8, 1, true>": 8 waves, conv a on waves
 * 0-3 and conv b on 4-7, a's activation handed over in LDS; the MFMA rows are the couts of both
 * output planes), the 16-channel steps on the D-streaming kernel with both convs' weights in every
 * wave; 2 = the split-wave kernel for both (PP for the 8 -> 8 steps); 1 = the split-wave kernel
 * without PP; 0 = the D-streaming kernel for both. */
int lea_conv3d_bf16_set_pair_split(int on);

/* Output words per thread of the c8 resample, k in {1, 2, 4}; 0 restores the default
 * (4 when up-sampling, else 1) (tools/resample_probe.py). */
int lea_resample_bf16_set_batch(int k);

/* c8 resample up-samplings: 1 (default) = the column-walking kernel (a wave walks R = 8 output
 * rows of 64 columns, each source row W-lerped once into registers, the next row's words
 * loaded one row ahead; "resample_c8_cols_kernel<8>"), 2 = the same with R = 16, 0 = the
 * per-output gather ("resample_c8_kernel<K>", also what a nonzero lea_resample_bf16_set_batch
 * selects).  Bit-identical. */
int lea_resample_bf16_set_cols(int on);

/* fp32 trilinear resample kernel: 0 (default) = the separable form where the output rows
 * are whole 16-byte words (W-lerped source rows in LDS), 1 = the row-staged form, 2 = the
 * per-output gather.  Bit-identical. */
int lea_resample_set_mode(int mode);

/* 1 (default) = lea_conv2d_bnrelu runs convs with cin <= 16 and cout <= 32 (the feature
 * net's cell ops) on the few-channel VALU tile ("conv2d_small_kernel<CIN4, NG>"), 0 = the
 * DMA / MFMA engine for every shape. */
int lea_conv2d_set_small(int on);

/* lea_conv2d_kernel_name with the input channel count (the few-channel tile depends on it). */
const char* lea_conv2d_kernel_name_cin(int B, int cin, int cout, int H, int W);

/* Disparity regression: 4 (default, r06) = form 3 (form 2 at D3 = 88) with D3 exponentials per
 * pixel instead of maxdisp (x3 depth up-sampling: exp(m - u) as products of exp((m - v_k) / 3);
 * within a few ulp per term of form 3, not bit-identical); 3 = the three-row staged kernel (one workgroup of 768
 * threads per three output rows: each raw source value loaded once; bit-identical to 2; D3 = 88
 * stays on 2); 2 (r05) = the row-staged kernel (a workgroup's two source
 * rows of every plane H-lerped into LDS, two passes over the planes, compile-time depth axis,
 * no rescaling softmin) for the configured (D3, maxdisp) pairs (4, 12), (8, 24), (16, 48),
 * (32, 96), (64, 192); 1 = the register kernel (D3 plane values in registers) for them; 0 = the
 * online-softmin kernel for every shape. */
int lea_disparity_set_register_form(int on);

/* Head tap-sum: 2 (default, r05) = passes 1 + 2 in one launch (a workgroup computes the
 * pass-1 values of its R output rows' low-res source rows straight into LDS; the workspace is
 * not touched), 1 = pass 1 through the workspace, then the row-staged pass 2 (R output rows'
 * low-res source rows of the 9 maps in LDS), each when those rows fit 64 KB; 0 = pass 1,
 * then one workgroup per output row gathering through the L1.  Identical bits. */
int lea_tapsum_set_rows(int on);

/* Host query (no GPU): the exact largest number of source rows a row-staged kernel's
 * workgroup reads when it owns R output rows plus `halo` rows either side, for a
 * trilinear axis Hi -> Ho (align_corners ac): the LDS bound of resample3d_rows/sep_f32
 * (halo 0) and tapsum_hwpass_rows_f32 (halo 1).  A kernel that ever met more rows than
 * this would write NaN rather than read rows it never staged.  Returns -1 (and sets
 * lea_last_error) on bad arguments: any positive value is a row count. */
int lea_staged_rows(int Hi, int Ho, int ac, int R, int halo);

/* 1 = the Winograd entries run 16-cout layers (the L1 cells' 16 -> 16 ops) on the F(2,3) along W
 * x F(2,3) along D tile with the packer's U and four waves per SIMD ("conv3d_wino22_kernel",
 * csrc/conv3d_wino22.hip); 0 = the F(4,3) x F(2,3) per-lane tile.  Same packed weights. */
int lea_conv3d_wino_set_w22(int on);

/* Winograd entries: tile override (np in {1, 2} tile rows per wave, td in {1, 2}
 * planes, f in {0 = planner, 2, 4, 8 = F(4,3) on 32-wide row pairs}; np = 0 resets;
 * depth-paired shapes keep np = 1, td = 2 and F(4,3)). */
int lea_conv3d_wino_set_tile_override(int np, int td, int f);

/* Engine variant for the Winograd entries (same packed weights): 0 = the planner's
 * choice, 1 = F(4,3) along W only, 2..4 = F(4,3) along W x F(2,3) along D
 * (csrc/conv3d_wino2.hip: "conv3d_wino2_kernel<Q, WC, MTE, NW, OCC, PV, CV>", PV 0 = per-lane V, 1/2 =
 * transform pass) where the cout block allows it (16 or 32 couts per block): 2 = four waves of one 16-row
 * cout tile, 3 = eight waves, 4 = two cout tiles per wave at one wave per SIMD. */
int lea_conv3d_wino_set_variant(int variant);

/* Depth pairs each W x D engine workgroup walks (its items = pairs x 4-channel chunks
 * through one DMA pipeline); 0 restores the planner. */
int lea_conv3d_wino2_set_walk(int spw);

/* 1 (default) = the W x D engine's transform-pass tiles stage their halo as 16-byte
 * LDS-DMA pieces where rows are whole 16-byte blocks (W % 4 == 0, aligned sources;
 * kernel name "..., 2, false>"), 0 = dword pieces ("..., 1, false>"). */
int lea_conv3d_wino2_set_halo16(int on);

/* The W x D engine's per-lane 16-cout tile: 2 (default) = 16-byte LDS-DMA halo pieces
 * in interleaved row sets (bank-conflict-free) with the fenced step schedule (kernel name
 * "conv3d_wino2_kernel<8, 1, 1, 4, 2, 5, false>"), 1 = the same halo with the compiler's
 * schedule ("..., 4, false>"), 0 = dword pieces ("..., 0, false>").  Bit-identical. */
int lea_conv3d_wino2_set_lane_halo16(int on);

/* 1 (default) = the 1-D engine's depth-paired 16-byte-halo tile (the L0 8 -> 8 cell ops)
 * issues each step's MFMAs as one block between sched_barriers (kernel name
 * "conv3d_wino_kernel<4, 16, 0, 1, 2, false, true, true>"), 0 = the compiler's interleaved
 * schedule ("..., false, true>").  Bit-identical. */
int lea_conv3d_wino_set_fence(int on);

/* 1 (default) = the 16-byte-halo W x D tile runs as the one-barrier pipeline
 * ("conv3d_wino2p_kernel": item i's MFMAs interleaved with item i + 1's transform pass,
 * weights loaded per lane from the packed buffer's per-lane copy), 0 = the two-barrier
 * tile (PV = 2).  Same packed weights. */
int lea_conv3d_wino2_set_pipeline(int on);

/* 1 (default since r06) = the pipelined W x D kernel reads the per-lane weights with G_W
 * already applied by the packer (54 floats per cout and channel; the step forms only the D
 * part of U: 197 -> 147 VALU per item, bit-identical outputs; -0.7 % per forward on the
 * kernel's layers, profiles/r06_wpre_ab.txt), 0 = the raw taps.  Both copies are always
 * packed. */
int lea_conv3d_wino2p_set_wpre(int on);

/* 2 (default since r06 v45) = as 1 and also the two-chunk layers (cin 8: the L0 8 -> 24 sibling
 * group; 275.6 -> 259.7 us, profiles/r06_w44_modes_ab.txt), 1 = the layers of the pipelined W x D
 * kernel run on the F(4,3) x F(4,3)
 * tile instead ("conv3d_wino44_kernel": 36 MFMA products per 4 x 4 outputs and kernel row
 * instead of 48; the W points split over two waves that swap accumulators in the epilogue;
 * -9.5 % on those layers, profiles/r06_w44_ab.txt), 0 = the pipelined F(4,3) x F(2,3)
 * kernel (the two-chunk layers then on the two-barrier tile), 3 = as 2 and the 16-cout layers as
 * half-empty 32-cout blocks.  Same packed weights (every per-lane copy is packed). */
int lea_conv3d_wino44_set(int on);

/* 1 = the F(4,3) x F(4,3) tile reads U itself from its per-lane copy (the packer applies both
 * G factors' matrices: 54 floats per cout, channel and x-half; the steps form no U), 0 = the
 * G_W' g copy with G_D' applied per step.  Bit-identical; both copies are always packed. */
int lea_conv3d_wino44_set_upre(int on);

/* Item-body schedule of the F(4,3) x F(4,3) tile (r06 A/B): 0 = the default (V-pass after the
 * first step's MFMAs, iglp_opt(0)), 1 = the V-pass after the second step's MFMAs, 2 = 0 without
 * iglp_opt, 3 = the V-pass after all MFMAs.  Bit-identical. */
int lea_conv3d_wino44_set_sched(int s);

/* The F(4,3) x F(4,3) tile's workgroup order: 0 = linear (cout block, depth group, tile),
 * g in 1..16 = groups of g x g tiles x max(1, 64 / (cout blocks g^2)) depth groups,
 * consecutive per XCD (L2 sharing of the halo), -1 (default) = 16 on grids of >= 2048
 * workgroups, else 0.  Bit-identical. */
int lea_conv3d_wino44_set_group(int g);

/* 1 (default) = the Winograd engines' buffer-addressed epilogue where the shape allows
 * it (W % 4 == 0, 16-B aligned output / residual; residual loads issued together, the
 * next chunk's DMA waited for without the stores), 0 = the per-group epilogue. */
int lea_conv3d_wino_set_epi_buf(int on);

/* couts <= 8 on the Winograd entries: 0 (default) = the depth-paired 1-D tile, 1 =
 * packed and planned as 16-row cout blocks (the W x D engine).  Packing and launches
 * must use the same mode. */
int lea_conv3d_wino_set_small_cout(int mode);

/* 48k-cout layers (not multiples of 32) on the Winograd entries: 1 (default) = 48-row
 * blocks of the 1-D engine, 0 = 32-row blocks of the W x D engine (last block padded).
 * Packing and launches must use the same setting. */
int lea_conv3d_wino_set_block48(int on);

#ifdef __cplusplus
}
#endif
#endif /* LEASTEREO_HIP_TUNING_H */
