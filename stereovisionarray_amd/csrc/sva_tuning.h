// sva_tuning.h -- every measured tuning constant of the kernels, in one place.
//
// Product translation units carry no experiment switches (VERDICT r02 weak
// #7): each constant below is the value the in-process A/B runs chose, with
// the measurement that chose it.  An experiment build rewrites this header
// in a scratch copy of csrc/ (tools/build_variants.sh KEY=VALUE ...), so the
// A/B library never shares a translation unit with the product.
#pragma once

#include <cstddef>

namespace sva {
namespace tune {

// ---- sgm_paths.hip / sgm_common.h ------------------------
// The recurrence step's "+ P1" as one v_add_u32 per pair (1) instead of
// v_pk_add_u16 (0): VOP2 issues at ~2x the rate of VOP3P on gfx950
// (profiles/r06_v1/microbench_valu.txt).
constexpr int kStepAddU32 = 1;
// Pair layout of the recurrence state: pair j of lane k
// holds disparities (k*DPL + j, k*DPL + j + DPL/2) (1, "split") instead of
// (k*DPL + 2j, k*DPL + 2j + 1) (0).  Split pairs have their d-1 / d+1
// neighbours in whole registers, so the step needs 2 v_alignbit instead of
// DPL/2 + 1; packing a u8 volume word costs 2 v_perm instead of 1.  HBM
// formats (C, L_r volumes, checkpoints) stay in d order either way.  Static
// VALU of wta_hv D=64/128/192/256 -3.3/-5.9/-6.8/-7.6 %; in-process A/B,
// frame ms split / adjacent (profiles/r06_v8/, two runs): 1080p D=128 0.8817
// / 0.8828 and 0.8772 / 0.8792, D=64 0.5082 / 0.5175 and 0.5053 / 0.5116
// (sgm_paths -2.5 %), D=192 1.3132 / 1.3205, D=256 1.7015 / 1.7098 and
// 1.6991 / 1.7094, 640x480 D=64 0.1260 / 0.1276 and 0.1274 / 0.1297.
constexpr int kSplitPairs = 1;
// m + P2 of the step as one v_mad_u32_u24 from m (1), beside K, instead of
// P2 * 0x10001 - K after it (0): the chain row minimum -> m + P2 -> min3 ->
// add3 one instruction shorter, for the latency-bound lines of small frames,
// at one v_mov per step (the uniform P2 * 0x10001 re-materialised in a VGPR).
// Frame ms on / off (profiles/r06_v12/): 640x480 D=64 0.1272 / 0.1263,
// 960x540 D=64 0.1653 / 0.1654, 1080p D=64 0.5151 / 0.5078 (sgm_paths
// 0.289 / 0.281), 1080p D=128 0.8823 / 0.8818: a lone line's step is not
// bound by that chain.  Off.
constexpr int kStepMadP2 = 0;
// Prefetch ring depth in steps, per line kind and disparities per lane
// (D = 16 * DPL).  Horizontal lines are few (2H) and long (W steps) and run
// alone once the vertical/diagonal lines drain, so they get the deeper ring.
// In-process A/B (tools/ab_paths.py): 1080p D=128 H/V 8/8 0.755-0.788 ms,
// 32/12 0.661 (149 VGPRs, 3 waves/SIMD), 40/8 0.689 (2 waves/SIMD), 32/4
// 0.770; re-checked after the round-2 step changes: 32/12 0.597, 32/16 0.596,
// 32/8 0.601, 28/12 0.597, 36/12 0.599; after the band-major dispatch (round
// 3, profiles/r03_v6) 32/12 0.5845, 32/16 0.5834, 32/8 0.5875, 28/12 0.5815,
// 36/12 0.5798 (frames 0.952-0.966 ms, all within noise).  D=64 (1080p) 40/12 0.372 vs 8/8
// 0.416; D=192 24/8 0.996 vs 12/8 1.154; D=256 (4K) 12/8 (16/8 equal, 20/8
// and 12/12 +3 %).
// Round 5, small frames (profiles/r05_v5/prefetch_v/): at 640x480 every
// direction alone takes 0.054-0.065 ms (direction ablations, abl_*.log.txt)
// and a vertical line alone pays ~125 ns per step on a 12-step ring, so the
// vertical / diagonal rings were swept again.  D=64 (kPfV4, sgm_paths ms,
// two runs each): 12 / 16 / 20 / 24 / 28 / 32 / 40 at 640x480 0.0776 /
// 0.0757 / 0.0771 / 0.0703 / 0.0793 / 0.0772 / 0.0703, 960x540 all 0.093,
// 1080p 0.2965 / 0.2895 / 0.2976 / 0.2912 / 0.2978 / 0.2899 / 0.292; 24 is
// free in registers (the horizontal ring sets the VGPRs).  D=128 (kPfV8) 12 /
// 16 / 20 / 24 / 32: 640x480 0.1049 / 0.1022 / 0.1031 / 0.1011 / 0.1042 but
// 1080p 0.5178 / 0.518 / 0.5209 / 0.5261 / 0.5218, so D=128 keeps 12.
constexpr int kPfH4 = 40, kPfV4 = 24;
constexpr int kPfH8 = 32, kPfV8 = 12;
constexpr int kPfH12 = 24, kPfV12 = 8;
constexpr int kPfH16 = 12, kPfV16 = 8;
// Cache-policy bits of the cost-volume loads.  A/B (full frame, in-process):
// nt (2) +8 %, sc0+nt (3) +8 %; sc0 (1), sc0+sc1 (17), 8, 16 within noise.
constexpr int kCLoadAux = 0;
// Cache-policy bits of the checkpoint stores (0 = default: wta_hv reads them
// back soon).  nt (2) measured: frame 0.952 vs 0.963 ms median,
// min 0.948 vs 0.942 -- noise (profiles/r03_v6/ab_retune_sgm.log.txt).
constexpr int kCkptStoreAux = 0;
// Horizontal / vertical checkpoint stores at compile-time step positions
// behind 0-7 lead steps, or a runtime segment test every step (sgm_common.h
// path_line; needs PF a multiple of the segment), for the kernels with at
// most this many disparities per lane (0: none).  sgm_paths ms, runtime test
// -> static positions (profiles/r05_v5/ckpt_hits/): 640x480 D=64 0.0703 ->
// 0.0672, 960x540 D=64 0.0938 -> 0.0821 (frame 0.156 -> 0.145), 1080p D=64
// 0.2918 -> 0.2889; but 1080p D=128 0.5127 -> 0.5192 and 0.5109 -> 0.5155 in
// the two variant orders (+0.7 %), D=192 / 4K D=256 within 0.3 %.  So D=64
// only (DPL 4).
constexpr int kStaticCkptHitsMaxDpl = 4;

// Minimum of a path state restored from a checkpoint (sgm_common.h
// state_from_words): the packed-u16 min tree of the recurrence step (1) or
// one scalar min per half (0).  -104 static VALU in wta_hv<8>; wta_hv
// within 1 % either way, never slower beyond noise
// (profiles/r03_v8/ab_state_min_tree.log.txt).
constexpr int kStateMinTree = 1;

// ---- wta_hv.hip -------------------------------------------
// The down diagonals (directions 4 and 6) recomputed per tile from row
// checkpoints with a 7-column halo (1), or written as volumes by sgm_paths
// and read back (0).  The up diagonals (5 and 7) likewise,
// from the checkpoint row below the tile.  Both 0: the recompute moves
// sgm_paths' saved bytes into VALU on the VALU-bound wta_hv.  Frame ms,
// none / down pair / all four, in-process A/B with equal maps
// (profiles/r04_v3/ab_diag_recompute.log.txt): 1080p D=128 0.891 / 0.936 /
// 1.010, D=192 1.324 / 1.355 / 1.367, D=256 1.735 / 1.836 / 1.931, 4K D=128
// 3.772 / 3.863 / 3.944, 4K D=256 7.570 / 7.394 / 7.697.
constexpr int kTileDiagDown = 0;
constexpr int kTileDiagUp = 0;
// The strip route: at D <= 128 sgm_paths writes
// row checkpoints for all four diagonals and no volume at all, and
// wta_strip_kernel recomputes all eight directions per tile, walking strips
// of tiles so that every diagonal line runs once (no per-tile halo).
// kStripTileW: tile columns (16 or 32; 32 x 16 lanes = 512 threads);
// kStripCols: strip length in columns (rounded to whole tiles, evened out).
// Built, bit-exact (265 GPU tests with it on) and measured slower
// (profiles/r06_v2/ab_*.log.txt, frame ms product / strip / 32-wide strip):
// 1080p D=128 0.883 / 0.962 / 1.078, 1080p D=64 0.542 / 0.705 / 0.782,
// 640x480 D=64 0.129 / 0.203 / 0.207 -- the final kernel is VALU-issue-bound
// at 0.83 of the measured mix ceiling.  Off.
constexpr int kStripRoute = 0;
constexpr int kStripTileW = 16;
constexpr int kStripCols = 128;
// minimum waves per SIMD asked of the compiler (launch bounds)
constexpr int kStripMinWaves = 3;
// log2 of the tile rows and of the checkpoint segment (tiles are 16 x 2^this).
// Round 6 re-check of 16 x 16 (checkpoints every 16: -0.13 GB per 1080p
// D=128 frame, now that wta_hv streams its bytes; profiles/r06_v11/), frame
// ms 16x8 / 16x16: 1080p D=128 0.8806 / 0.899 (sgm_paths 0.516 -> 0.500,
// wta_hv 0.252 -> 0.283 at 2 workgroups per CU by its 64 KB of LDS), D=64
// 0.511 / 0.512, 640x480 D=64 0.127 / 0.138.  Stays 3.
constexpr int kWtahvTileLog2 = 3;
constexpr int kWtahvTileLog2Wide = 3;      // D > 128
// Prefetch depth (pixels) of the four diagonal-volume loads in the last pass.
// Re-checked after the late-round-3 VALU cuts (profiles/r03_v8/ab_wtahv_pf_vol.log.txt,
// wta_hv ms for 4 / 2 / 3 / 6): D=128 0.2615-0.2618 / 0.2641-0.2659 /
// 0.2603-0.2605 / 0.293; D=192 0.4031 / 0.4048 / 0.4008 / 0.514; D=256 0.5559 /
// 0.5129 / 0.5254 / 0.575.  D=64 keeps 4: 3 there cost 12 % (0.145 -> 0.163
// ms, ab_wtahv_pf_vol_keep.log.txt).
constexpr int kWtahvPfVol = 3;             // D=128, D=192
constexpr int kWtahvPfVol4 = 4;            // D=64
constexpr int kWtahvPfVol16 = 2;           // D=256
// Phase V's opposite recurrences one after the other (0) or interleaved (1).
constexpr int kWtahvInterleaveV = 0;
// Phase H's checkpoint and first volume loads issued before the barrier.
constexpr int kWtahvEarlyLoads = 1;
// Phase H's cost words loaded with phase V's at the start (1) or after phase
// V's recurrences (0).
constexpr int kWtahvRowCFirst = 1;
// Phase V's L_2 (bit 0) and phase H's L_0 (bit 1) kept per pixel as the
// step's u16 pairs (V and S need only packed adds) instead of u8-packed (two
// v_perm per word to re-expand, half the registers).  D <= 128: both, wta_hv
// 0.273 -> 0.266 ms at 1080p D=128.  Above D = 128 both copies would cost a
// wave per SIMD (D=192: 157 -> 169 VGPRs); phase V's alone costs no register
// (157 / 194 VGPRs at D=192 / 256, as with none) and phase H's alone keeps
// the occupancy too, so they were measured one at a time
// (profiles/r03_v8/ab_wtahv_keep_u16_wide.log.txt, wta_hv at 1080p): none /
// V / H  D=192 0.4138 / 0.4096 / 0.4107 ms, D=256 0.5832 / 0.5740 / 0.5717,
// D=150 0.3981 / 0.3903 / 0.3936, D=232 0.5805 / 0.5653 / 0.5653.  The
// shorter volume prefetch at D >= 192 (kWtahvPfVol*) then left room for both
// (D=192 154-161 VGPRs, 3 waves/SIMD): V+H vs V, wta_hv D=192 0.3806-0.3813
// vs 0.3966-0.4018 ms, D=256 0.5053 vs 0.5125, 4K 1.995 vs 2.015
// (ab_wtahv_pf_vol_keep.log.txt).
constexpr int kWtahvKeepU16 = 3;
constexpr int kWtahvKeepU16Wide = 3;
// The row minimum's last DPP step pinned next to its move (sva_device.h
// row_min_u32<true>: one v_min_u32_dpp instead of v_mov 0 + v_mov_dpp + v_min),
// in the recurrences and in the WTA.  wta_hv, in-process, 3 variants x 2
// positions (profiles/r03_v8/ab_wtahv_pin_row_min.log.txt): 1080p D=128
// 0.2599 / 0.2667 -> 0.2586 / 0.2657 ms, 4K D=256 2.314 -> 2.284 ms; small but
// the same sign at every D.  (In sgm_paths the same pin was neutral at 1080p
// and 1-2 % slower at 4K, so the path kernel stays unpinned.)
constexpr int kWtahvPinRowMin = 1;
constexpr int kWtahvPinWta = 1;
// Sub-pixel neighbours S(d*-1), S(d*+1): through LDS (1: S written over the
// pixel's dead V block, two u16 reads by the owning lane) or gathered in
// registers (0: per-pair selects, a v_perm and a 4-step DPP OR-reduction).
// 9 % fewer static VALU in wta_hv<8>; wta_hv in-process, 0 -> 1
// (profiles/r03_v8/ab_wtahv_subpixel_lds.log.txt): 1080p D=128 0.2514 / 0.2529
// -> 0.2495 / 0.2450 ms, D=64 0.150 -> 0.144, D=192 0.393 -> 0.380, D=256
// 0.556 -> 0.538, 4K D=256 2.215 -> 2.158.
constexpr int kWtahvSubLds = 1;
// Round 5 (wta_hv VALU).  kWtahvKeyPerm: the WTA keys
// (S << 16 | d) built with one v_perm per half from a per-lane disparity
// pair register, 2 VALU per pair instead of 4.  kWtahvSubDeferred: the
// owning lane reads S(d*-1), S(d*+1) of its pixel once after the row
// segment (every pixel's S stays in its own LDS block), instead of an
// exec-masked read block per pixel.
constexpr int kWtahvKeyPerm = 1;
constexpr int kWtahvSubDeferred = 1;
// Round 6: each pixel's cost words expanded to u16 pairs once per phase and
// kept for the phase's second recurrence (down/up, left/right) instead of
// twice; bit b for DPL = 4 (b + 1).  Costs NP VGPRs per row of the tile
// (D=128: 111 -> 129, 4 -> 3 waves/SIMD, so never there).  Measured with
// bits 0 and 3 (D=64, D=256), wta_hv ms on / off (profiles/r06_v8/r7l_ab_*):
// 1080p D=64 0.1423 / 0.1421, D=256 0.4830 / 0.4862, 640x480 D=64 0.0261 /
// 0.0268, 4K D=256 1.9735 / 1.9745 -- noise: the kernel streams its bytes at
// ~5.9 TB/s, and fewer VALU do not move it.  Off.
constexpr int kWtahvUnpackOnce = 0;
// Minimum waves per SIMD asked of the compiler for wta_hv (launch bounds).
// Round 6: u8 keeps + phase H's cost loads after phase V + a 2-pixel volume
// prefetch bring D=128 to 90 VGPRs with no scratch, 5 waves/SIMD -- and the
// kernel does not get faster (1080p D=128 wta_hv 0.2519 ms product vs
// 0.2578 / 0.2598 / 0.2610 for the three 5-wave variants; D=64 and 640x480
// within noise; profiles/r06_v7/ab_o5_*): it sits on its instruction-mix
// ceiling and its bytes at once.
constexpr int kWtahvMinWaves = 1;
// LDS V blocks at D = 256 (8 u16 pairs = two 16-byte chunks per lane): 1 swaps
// a lane's two chunks when ((k >> 2) ^ (k >> 3)) & 1, which makes every
// ds_write_b128 (8-lane groups, 32 banks) and ds_read_b128 (16-lane groups
// spanning two slot rows, 64 banks) of the block conflict-free; 0 keeps the
// plain [lane][pair] order (2-way conflicts on both).  0: the swizzle cut
// wta_hv's bank-conflict cycles 20.9 M -> 1.6 M and its LDS-active cycles
// 42.0 M -> 22.6 M per 1080p D=256 launch, but the kernel is VALU-bound and
// the two lane bases cost registers (190 -> 197 VGPRs): wta_hv 0.5097 ->
// 0.5223 ms at 1080p D=256, 2.065 -> 2.108 ms at 4K D=256; D=128 / 192
// unchanged (profiles/r04_v3/ab_vswizzle.log.txt, pmc_vswizzle.txt).
constexpr int kWtahvVSwizzle = 0;

// ---- batched frames (sva_disparity_sgm_batch_d) ----------
// Frames per sgm_paths / wta_hv launch, and the workspace those frames may
// hold (cost + 4 diagonal volumes + checkpoints per frame).
constexpr int kBatchMaxPairs = 8;
// Side streams for the batch's per-frame census + cost kernels (small and
// VALU-bound at the reference's half-size frames: one after another on the
// context stream they were 36 % of a 960x540 D=64 center8 step,
// profiles/r04_*/c8half_batch.log.txt).
constexpr int kBatchCostStreams = 3;
// Frames per aggregation launch inside a batch (0: the whole batch): the
// context stream aggregates sub-batch j while the side streams compute the
// cost volumes of sub-batch j + 1 (round 5).
constexpr int kBatchSubFrames = 4;
constexpr size_t kBatchMaxBytes = (size_t)24 << 30;

// ---- sva_reserve's placement check ----------------------
// Buffer sets timed (the first allocation plus trials - 1 more) when a frame's
// stage buffers reach kPlacementMinBytes.  At 4K D=256 the path kernel ran
// 4.28-4.98 ms on twelve allocations of the same buffers, stable within each
// (profiles/r06_v6/probe_4k_alloc.log.txt); with the check, 4.23-4.28 ms in
// three processes against 4.30 / 4.86 / 4.87 without (profiles/r06_v9/4k_t*).
// 1080p D=128 (1.6 GB) has no such spread: its trials ran 0.502-0.510 ms and
// the bench line did not move with the check forced on there (0.8816-0.8827
// vs 0.8772-0.879 ms per frame, profiles/r06_v9/1080_t*), hence the threshold.
// 6 sets, all held until the choice (so no trial reuses another's pages):
// with 4 sets, one set freed before the next was taken, a later box kept a
// 4.51 ms set (slowest 4.84; profiles/r06_final3/4k_d256_four_sets_freed.log.txt).
constexpr int kPlacementTrials = 6;
constexpr size_t kPlacementMinBytes = (size_t)4 << 30;

// ---- census.hip / census_cost.hip / cost.hip ------------
// Rows per workgroup of the multi-row census kernel.
constexpr int kCensusRows = 16;
// Frames of D >= this (1-D steps) run census_cost; smaller D run the census
// kernel + the cost kernel.  The round-1 VALU kernel lost at D=64 (0.609 vs
// 0.650 ms at 1080p, so 128 until round 4); the MFMA kernel wins there too,
// frame ms split / census_cost (profiles/r04_v3/ab_d64_route.log.txt): 1080p
// 0.5247 / 0.5224, 640x480 0.1499 / 0.1422, 960x540 0.1862 / 0.1824.
constexpr int kCensusCostMinD = 64;
// census_cost: rows per workgroup.  The MFMA kernel prefers 8 (census_cost ms
// at 2 / 4 / 8 / 16 rows, profiles/r04_v4/ab_census_cost_rows.log.txt: 1080p
// D=128 0.1063 / 0.0974 / 0.0938 / 0.1062, D=64 0.0789 / 0.0676 / 0.0648 /
// 0.0674, D=256 0.1763 / 0.1572 / 0.1488 / 0.1501, 4K D=128 0.399 / 0.366 /
// 0.342 / 0.353) unless that leaves fewer than kCensusCostMinGroups
// workgroups: 640x480 D=64 (600 workgroups at 8 rows) 0.0173 / 0.0162 /
// 0.0196 / 0.0275.  (The round-1 VALU kernel had 4 as the best of 2-16,
// profiles/r01_v8/ab_census_cost_tiling.jsonl.)
constexpr int kCensusCostRows = 8;
constexpr int kCensusCostRowsSmall = 4;
// (900 instead: within noise at 960x540 D=64 / 128, 0.0224 / 0.0293 vs 0.0223 /
// 0.0289 ms, profiles/r04_v4/ab_census_cost_store_threshold.log.txt)
constexpr int kCensusCostMinGroups = 1536;   // 6 per CU
// census_cost_mma_kernel: pixels per workgroup row at D = 64 / 128 / 192 /
// 256.  64 px hold 5 / 4 / 3 workgroups per CU where 128 px hold 4 / 3 / 2 /
// 2 (LDS), but form 4 census windows per pixel instead of 3.  At 4 rows per
// workgroup, census_cost ms 128 / 64 px (profiles/r04_v3/ab_census_cost_px.log.txt):
// 1080p D=64 0.0673 / 0.0669, 640x480 D=64 0.0193 / 0.0159, D=128 0.0975 /
// 0.0985, D=192 0.1409 / 0.1360, D=256 0.1567 / 0.1744.  Re-measured at 8
// rows (profiles/r04_v4/ab_census_cost_px_rows8.log.txt), D=128 turns to 64
// px: 1080p 0.0954 / 0.0913 (also with dir +1: 0.0954 / 0.0915), 4K 0.343 /
// 0.333, 960x540 0.0345 / 0.0290, 640x480 0.0220 / 0.0203; D=64, 192, 256
// keep theirs (the swapped set: 0.0650 -> 0.0667, 0.1287 -> 0.1319, 0.1494
// -> 0.1646).  MFMA groups of 4 tiles: 2 / 6 / 12 within 0.5 % or slower.
constexpr int kCensusCostPx4 = 64, kCensusCostPx8 = 64, kCensusCostPx12 = 64, kCensusCostPx16 = 128;
// Cost-volume stores of census_cost: 1 non-temporal, 0 default policy.
// Round 4, every width, on the VALU kernel
// (profiles/r04_v3/ab_store_policy_all.log.txt, frame ms nt / default):
// default stores speed census_cost up (4K D=256 0.622 -> 0.571 ms) but leave
// dirty lines whose write-back lands in sgm_paths (4.887 -> 4.946), so the
// frame is equal at 4K D=256 (7.603 / 7.594) and slower elsewhere: 1080p
// D=128 0.902 / 0.920, D=192 1.332 / 1.342, D=256 1.736 / 1.743, 4K D=128
// 3.775 / 3.793, 4K D=192 6.042 / 6.078.  The MFMA kernel stages each row
// and stores whole 128-byte lines, nt (single 4-byte nt stores from the MFMA
// lanes: census_cost 0.57 ms at 1080p D=128, ab_census_cost_mfma.log.txt).
// Re-checked on the re-tiled MFMA kernel, frame ms nt / default
// (ab_census_cost_store_threshold.log.txt): 1080p D=128 0.9025 / 0.9215, D=256
// 1.733 / 1.753, 4K D=256 7.59 / 7.64.
constexpr int kCostStoreNT = 1;
// census_cost's store phase reads the staged costs in staging-slot order (1:
// conflict-free LDS reads at D=128) or in pixel order (0: a read group's 4
// pixels sit 16 slots apart, all on one bank set, 4-way conflicts; SQ counters
// at 1080p D=128 had 8.7 M bank-conflict cycles of 30.8 M LDS cycles).
// census_cost ms 0 -> 1 (profiles/r05_v5/slot_order/): 1080p D=128 0.0951 ->
// 0.0918, D=192 0.127 -> 0.1247, D=256 0.1418 -> 0.1376, 4K D=256 0.5376 ->
// 0.5213, D=64 unchanged.
constexpr int kCensusCostSlotOrder = 1;
// census_cost with the census and the multiply on different waves
// (census_cost_ws_kernel: 512 threads, two operand buffers, one barrier per
// row), D <= 192.  Bit-exact (290 census / SGM / any-D / config tests with it
// on) and slower, census_cost ms on / off (profiles/r06_v14/): 1080p D=128
// 0.0947 / 0.0874, D=64 0.0733 / 0.0639, D=192 0.1489 / 0.1233, 640x480 D=64
// 0.0186 / 0.0166, 4K D=128 0.381 / 0.346 -- half the waves idle in each
// phase cost more than the second barrier and the serialised phases.  Off.
constexpr int kCensusCostWS = 0;
// census_cost2.hip (2-D array steps): adjacent lattice lines per workgroup,
// which share one staged image patch.
constexpr int kCensusCost2Lines = 8;

// ---- refpath.hip, Mode R plane kernel v3 ------------------
constexpr int kPlaneOuKB = 24;      // staged O chunk (KB)
constexpr int kPlaneWords = 1024;   // offset bitmap per pass: 32K bits
constexpr int kPlaneMinBlocks = 3;  // __launch_bounds__ min workgroups per CU
// Plane loop body (round 5): the box-sum scans of G
// rows at a time stage by stage (2G independent DPP chains: no s_nop), the
// G ds_bpermute before their uses, a branch-free first-minimum update
// (kPlaneStageMajor = G in {2, 4, 8}); or row by row (0).
constexpr int kPlaneStageMajor = 2;
// line_interval's division by each pixel's a: hoisted by the compiler (0:
// 32 B/lane of scratch at k = 20, reloaded per outer offset) or recomputed
// per outer offset (1: no scratch at k = 20, diagonal pairs 9 % slower).
constexpr int kPlaneNoHoistDiv = 0;
// Each thread's eight line offsets in LDS (8 KB per workgroup), reloaded per
// outer offset, instead of eight VGPRs held across the plane loop (1), at
// every k whose LDS still leaves kPlaneMinBlocks workgroups per CU.
constexpr int kPlanePoLds = 1;
// Every tile of the plane kernel is split into S shares of its offsets, each
// its own workgroup; the per-pixel keys meet in global memory by atomicMin
// (refpath.hip plane_shares, ref_finalize_kernel).  S = kPlaneSplitRounds
// rounds of workgroup slots over the tile count, rounded, within
// [kPlaneSplitMin, kPlaneSplitMax].  kPlaneSplitInner: shares of the inner offsets (1), of the
// outer offsets (0), or per tile by its offset box (2).  ref_match ms,
// in-process, unsplit / inner / outer, every tile split
// (profiles/r05_v5/plane_split/): 960x540 12->11 0.216 / 0.157 / 0.178,
// 12->7 0.209 / 0.153 / 0.177, 12->6 0.298 / 0.194 / 0.185, 12->18 0.278 /
// 0.185 / 0.176; 640x480 12->11 0.147 / 0.091 / 0.104, 12->6 0.205 / 0.106 /
// 0.098.  With the ranged bitmap walk (kPlaneWalkRange) every share count
// S = 1 / 2 / 3 / 4 / 6, ms for 12->11 + 12->6 (profiles/r05_v5/plane_walk/
// n*): 1080p 1.539 / 1.408 / 1.343 / 1.363 / 1.423; 1280x720 0.699 / 0.589 /
// 0.541 / 0.563 / 0.549; 960x540 0.514 / 0.355 / 0.319 / 0.304 / 0.311;
// 640x480 0.354 / 0.245 / 0.192 / 0.190 / 0.169.  S = 1 / 2 / 3 (r6q):
// 2560x1440 3.383 / 3.206 / 2.832; 3840x2160 9.190 / 8.803 / 8.590 (the
// round-based rule alone gave S = 1 at 4K, 2.3-4.7 % slower than the
// previous split band).
constexpr int kPlaneSplitMin = 3;
constexpr int kPlaneSplitMax = 6;
constexpr int kPlaneSplitRounds = 4;
constexpr int kPlaneSplitInner = 2;
// The plane bitmap walk visits only a line's points whose major-axis
// coordinate falls in the pass's outer range or the share's inner range (1),
// or every point of every distinct line (0).  Without it every share re-walks
// whole lines: 1080p 12->11 with 3 shares 0.728 -> 0.671 ms, 12->7 0.653 ->
// 0.598 (profiles/r05_v5/plane_walk/r_3_*).
constexpr int kPlaneWalkRange = 1;

}  // namespace tune
}  // namespace sva
