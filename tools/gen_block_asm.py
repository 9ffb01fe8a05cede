#!/usr/bin/env python3
"""Generate anyseq_amd/csrc/anyseq_block_asm.inc: the hand-scheduled 32-step
steady-state block of the fill kernel (R = 1, X = 0, CH = 32) as inline-asm
strings, one per value space (G: global/semiglobal, L: local).

Per step (all lanes live):  C v_cmp_eq_u32_sdwa vcc, q, s.byte   substitution test
                            D v_cndmask_b32     w, wx, wm, vcc   weight
                            E v_add_u32         a, dg, w         diag + weight
                            A v_mov_b32_dpp     T, cur wave_shr:1  up (lane 0 keeps T = top row)
                            B v_max3_i32        O, a, cur, T     cell
(L adds  v_sub_u32 O, O, ng clamp  and  v_max_i32 best, best, O.)
The DPP reads `cur` written >= 3 instructions earlier (the VALU->DPP hazard needs
2), and writes in place into the register holding the top-row value, so a step is
five VALU with no copies and no stalls.

Registers: the 32 top-row values T0..T31 and the 32 cell values O0..O31 of the
block live in fixed VGPRs (clobbered); the top row comes in with eight broadcast
ds_read_b128.  Lane 63's bottom row leaves through a DPP shift register: once
O(u-1) is dead (after step u), `v_mov_b32_dpp O(u-1), O(u-2) wave_shl:1` moves
the register down one lane while lane 63 keeps its own cell, so after the block
lanes 32..63 of O31 hold lane 63's 32 cells in column order and ONE ds_write_b32
(per-lane address `pa`, lanes 0..31 into a dummy slot) publishes them.  A wide
store from a single lane would cost ~29 issue cycles per ds_write_b128 plus exec
switches; the shift costs one VALU per step off the critical path.
"""
import os
import sys

T0, O0, W, A = 64, 96, 128, 129   # fixed VGPRs: T 64..95, O 96..127, w, a (<= 170 VGPRs: 3 waves/SIMD)


def v(n):
    return f"v{n}"


def gen(kind, reads=True, stores=True, store_mode="shift"):
    L = kind == "L"
    out = []
    e = out.append
    # top row of this block: T0..T31 = ring[ra + 0 .. 124]
    for i in range(8):
        if reads:
            e(f"ds_read_b128 v[{T0 + 4 * i}:{T0 + 4 * i + 3}], %[ra] offset:{16 * i}")
    if reads:
        e("s_waitcnt lgkmcnt(6)")          # T0..T7 landed
    cur = "%[cur]"
    dg = "%[dg]"
    for u in range(32):
        c = u // 8
        if u % 8 == 0 and c >= 1 and stores and store_mode != "shift":
            # lane 63 publishes chunk c-1's eight cells (two b128 stores) before the
            # first step of chunk c; exec is restored >= 5 instructions before the next DPP
            o = O0 + 8 * (c - 1)
            if store_mode == "exec":
                e("s_mov_b64 %[sv], exec")
                e("s_mov_b64 exec, %[pm]")
            if store_mode != "exec_only":
                e(f"ds_write_b128 %[pa], v[{o}:{o + 3}] offset:{32 * (c - 1)}")
                e(f"ds_write_b128 %[pa], v[{o + 4}:{o + 7}] offset:{32 * (c - 1) + 16}")
            if store_mode in ("exec", "exec_only"):
                if store_mode == "exec_only":
                    e("s_mov_b64 %[sv], exec")
                    e("s_mov_b64 exec, %[pm]")
                e("s_mov_b64 exec, %[sv]")
                e("s_nop 1")
        if u % 8 == 0 and c >= 1 and reads:
            # chunk c reads T(8c-1)..T(8c+6), i.e. b128 reads up to r = (8c+6)//4; the
            # 7-r younger reads and the 2c stores issued so far may stay in flight
            r = (8 * c + 6) // 4
            e(f"s_waitcnt lgkmcnt({7 - r + (2 * c if stores and store_mode != 'shift' else 0)})")
        s = f"%[s{u // 4}]"
        b = u % 4
        tv = "%[tf]" if u == 0 else v(T0 + u - 1)
        ov = v(O0 + u)
        e(f"v_cmp_eq_u32_sdwa vcc, %[q], {s} src0_sel:DWORD src1_sel:BYTE_{b}")
        e(f"v_cndmask_b32_e32 v{W}, %[wx], %[wm], vcc")
        e(f"v_add_u32_e32 v{A}, {dg}, v{W}")
        e(f"v_mov_b32_dpp {tv}, {cur} wave_shr:1 row_mask:0xf bank_mask:0xf")
        e(f"v_max3_i32 {ov}, v{A}, {cur}, {tv}")
        if L:
            e(f"v_sub_u32_e64 {ov}, {ov}, %[ng] clamp")
            e(f"v_max_i32_e32 %[best], %[best], {ov}")
        if stores and store_mode == "shift" and u >= 2:
            # O(u-1) is dead now: shift register step (lane 63 keeps its cell)
            e(f"v_mov_b32_dpp {v(O0 + u - 1)}, {v(O0 + u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
        cur = ov
        dg = tv
    # last chunk's cells, then the block outputs
    o = O0 + 24
    if stores and store_mode == "shift":
        e(f"v_mov_b32_e32 %[cur], v{O0 + 31}")
        e(f"v_mov_b32_e32 %[dg], v{T0 + 30}")
        e(f"v_mov_b32_dpp {v(O0 + 31)}, {v(O0 + 30)} wave_shl:1 row_mask:0xf bank_mask:0xf")
        e(f"v_mov_b32_e32 %[tf], v{T0 + 31}")
        e("s_nop 1")
        e(f"ds_write_b32 %[pa], {v(O0 + 31)}")
        return out
    if stores:
        if store_mode in ("exec", "exec_only"):
            e("s_mov_b64 %[sv], exec")
            e("s_mov_b64 exec, %[pm]")
        if store_mode != "exec_only":
            e(f"ds_write_b128 %[pa], v[{o}:{o + 3}] offset:96")
            e(f"ds_write_b128 %[pa], v[{o + 4}:{o + 7}] offset:112")
        if store_mode in ("exec", "exec_only"):
            e("s_mov_b64 exec, %[sv]")
    e(f"v_mov_b32_e32 %[cur], v{O0 + 31}")
    e(f"v_mov_b32_e32 %[dg], v{T0 + 30}")
    e(f"v_mov_b32_e32 %[tf], v{T0 + 31}")
    return out

# s_sleep between polls of an LDS counter (0: spin); ANYSEQ_GEN_SLEEP overrides (experiments)
SLEEP = int(os.environ.get("ANYSEQ_GEN_SLEEP", "1"))
SK0, VT, VT2, VA, VB = 130, 138, 139, 140, 141   # subject words, temps, LDS addresses
TA, TB = 96, 98                                   # fixed SGPR pairs for s_memrealtime


def wait(e, name, seen, target, addr, count=None, tmp=None, signed=False):
    """Spin until seen >= target, refreshing `seen` from the LDS word at `addr`
    (wave-uniform), with s_sleep between polls.  The 10 s s_memrealtime limit
    starts at the 256th poll and is checked every 256 polls (-> L_timeout): the
    common case (ready within a few polls) issues no SMEM read, whose latency the
    poll's lgkmcnt(0) would otherwise wait for on the hand-off's critical path."""
    cmp = "s_cmp_ge_i32" if signed else "s_cmp_ge_u32"
    e(f"{cmp} {seen}, {target}")
    e(f"s_cbranch_scc1 L_{name}_ok_%=")
    e("s_mov_b32 %[x3], 0")
    e(f"L_{name}_loop_%=:")
    tmp = VT2 if tmp is None else tmp
    e(f"ds_read_b32 v{tmp}, {addr}")
    e("s_waitcnt lgkmcnt(0)")
    e(f"v_readfirstlane_b32 {seen}, v{tmp}")
    e(f"{cmp} {seen}, {target}")
    e(f"s_cbranch_scc1 L_{name}_ok_%=")
    if count:
        e(f"s_add_u32 {count}, {count}, 1")
    if SLEEP:
        e(f"s_sleep {SLEEP}")
    e("s_add_u32 %[x3], %[x3], 1")
    e("s_and_b32 %[x2], %[x3], 255")
    e(f"s_cbranch_scc1 L_{name}_loop_%=")
    e("s_cmp_eq_u32 %[x3], 256")
    e(f"s_cbranch_scc0 L_{name}_chk_%=")
    e(f"s_memrealtime s[{TA}:{TA + 1}]")
    e("s_waitcnt lgkmcnt(0)")
    e(f"s_branch L_{name}_loop_%=")
    e(f"L_{name}_chk_%=:")
    e(f"s_memrealtime s[{TB}:{TB + 1}]")
    e("s_waitcnt lgkmcnt(0)")
    e(f"s_sub_u32 s{TB}, s{TB}, s{TA}")
    e(f"s_subb_u32 s{TB + 1}, s{TB + 1}, s{TA + 1}")
    e(f"s_cmp_lg_u32 s{TB + 1}, 0")
    e("s_cbranch_scc1 L_timeout_%=")
    e(f"s_cmp_gt_u32 s{TB}, 1000000000")
    e("s_cbranch_scc1 L_timeout_%=")
    e(f"s_branch L_{name}_loop_%=")
    e(f"L_{name}_ok_%=:")


SKB_ = 142   # second subject-word set (double buffer): v142..v149


def throttle(e, k):
    """Band 0 of a problem (the only band that waits for nothing) sleeps %[thr]
    s_sleep-1 units per block: the chain then runs at band 0's slightly slower
    pace, and every later band has slack to absorb its hand-off jitter instead of
    adding it to the chain."""
    e("s_mov_b32 %[x2], %[thr]")
    e(f"L_thr{k}_%=:")
    e("s_cmp_eq_u32 %[x2], 0")
    e(f"s_cbranch_scc1 L_thrd{k}_%=")
    e("s_sleep 1")
    e("s_sub_u32 %[x2], %[x2], 1")
    e(f"s_branch L_thr{k}_%=")
    e(f"L_thrd{k}_%=:")


def gen_loop2(kind, border, pub, ts=False):
    """Steady-state loop specialised by role (no per-block flag tests):
    border: band 0 writes the scheme's top border into its own ring;
    pub: "lds" (next band of the group), "glob" (the group's last band: the
    next group's row buffer or out_row, plus the tail counter) or "none" (last
    band of the problem without an output row; reports tail).
    The subject words of block b+1 are prefetched during block b into the other
    of two register sets (the body is unrolled twice)."""
    L = kind == "L"
    trailing = pub != "lds"
    out = []
    e = out.append
    sets = (SK0, SKB_)

    def body(k):
        cs, ns = sets[k], sets[1 - k]
        e("s_add_u32 %[x1], %[b], 1")
        # prefetch the next block's subject words
        e("s_cmp_ge_u32 %[x1], %[be]")
        e(f"s_cbranch_scc1 L_nopf{k}_%=")
        e("s_add_u32 %[x4], %[b], 2")
        wait(e, f"sf{k}", "%[sf]", "%[x4]", "%[asf]", "%[nsf]" if ts else None)
        e("s_and_b32 %[x2], %[x1], 31")
        e("s_lshl_b32 %[x2], %[x2], 11")
        e(f"v_add_u32_e32 v{VA}, %[x2], %[skb]")
        for i in range(4):
            e(f"ds_read2st64_b32 v[{ns + 2 * i}:{ns + 2 * i + 1}], v{VA} offset0:{2 * i} offset1:{2 * i + 1}")
        e(f"L_nopf{k}_%=:")
        # top row of block b
        if border:
            e("s_lshl_b32 %[x0], %[b], 5")
            e("s_mul_i32 %[x2], %[x0], %[bvs]")
            e(f"v_add_u32_e32 v{VT}, %[x2], %[bvb]")
            e("s_lshl_b32 %[x2], %[x0], 2")
            e(f"v_add_u32_e32 v{VT2}, %[x2], %[lid4]")
            e(f"v_and_b32_e32 v{VT2}, 0x7ff, v{VT2}")
            e(f"v_add_u32_e32 v{VT2}, %[rb], v{VT2}")
            e(f"ds_write_b32 v{VT2}, v{VT}")
            throttle(e, k)
        else:
            wait(e, f"pr{k}", "%[sp]", "%[x1]", "%[apr]", "%[npr]" if ts else None)
        if ts:
            e("s_cmp_lg_u32 %[b], 0")
            e(f"s_cbranch_scc1 L_nots{k}_%=")
            e("s_memrealtime %[ts]")
            e("s_waitcnt lgkmcnt(0)")
            e(f"L_nots{k}_%=:")
        if pub == "lds":
            # chunk b-2 goes to slot (b-2) & 15: free once the consumer is at >= b-17
            e("s_cmp_lt_u32 %[b], 17")
            e(f"s_cbranch_scc1 L_nobp{k}_%=")
            e("s_sub_u32 %[x4], %[b], 17")
            wait(e, f"bp{k}", "%[sc]", "%[x4]", "%[anc]", "%[nbp]" if ts else None)
            e(f"L_nobp{k}_%=:")
        e("s_lshl_b32 %[x2], %[b], 7")
        e("s_and_b32 %[x2], %[x2], 2047")
        e("s_add_u32 %[x2], %[x2], %[rb]")
        e(f"v_mov_b32_e32 v{VB}, %[x2]")
        for i in range(8):
            e(f"ds_read_b128 v[{T0 + 4 * i}:{T0 + 4 * i + 3}], v{VB} offset:{16 * i}")
        cur, dg = "%[cur]", "%[dg]"
        for u in range(32):
            c = u // 8
            if u % 8 == 0:
                r = (8 * c + 6) // 4
                e(f"s_waitcnt lgkmcnt({7 - r})")
            sw = v(cs + u // 4)
            tv = "%[tf]" if u == 0 else v(T0 + u - 1)
            ov = v(O0 + u)
            e(f"v_cmp_eq_u32_sdwa vcc, %[q], {sw} src0_sel:DWORD src1_sel:BYTE_{u % 4}")
            e(f"v_cndmask_b32_e32 v{W}, %[wx], %[wm], vcc")
            e(f"v_add_u32_e32 v{A}, {dg}, v{W}")
            e(f"v_mov_b32_dpp {tv}, {cur} wave_shr:1 row_mask:0xf bank_mask:0xf")
            e(f"v_max3_i32 {ov}, v{A}, {cur}, {tv}")
            if L:
                e(f"v_sub_u32_e64 {ov}, {ov}, %[ng] clamp")
                e(f"v_max_i32_e32 %[best], %[best], {ov}")
            if u >= 2 and pub != "none":
                e(f"v_mov_b32_dpp {v(O0 + u - 1)}, {v(O0 + u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
            cur, dg = ov, tv
        e(f"v_mov_b32_e32 %[cur], v{O0 + 31}")
        e(f"v_mov_b32_e32 %[dg], v{T0 + 30}")
        if pub != "none":
            e(f"v_mov_b32_dpp {v(O0 + 31)}, {v(O0 + 30)} wave_shl:1 row_mask:0xf bank_mask:0xf")
        e(f"v_mov_b32_e32 %[tf], v{T0 + 31}")
        if pub != "none":
            e("s_cmp_lt_u32 %[b], 2")
            e(f"s_cbranch_scc1 L_nopub{k}_%=")
            e("s_sub_u32 %[x2], %[b], 2")
            e("s_lshl_b32 %[x2], %[x2], 7")
            if pub == "lds":
                e("s_and_b32 %[x2], %[x2], 2047")
                e("s_add_u32 %[x2], %[x2], %[nb]")
            e(f"v_add_u32_e32 v{VT}, %[x2], %[lo]")
            e("s_mov_b64 s[%d:%d], exec" % (TA, TA + 1))
            e("s_mov_b64 exec, %[hm]")
            if pub == "lds":
                e(f"ds_write_b32 v{VT}, v{O0 + 31}")
            else:
                e(f"global_store_dword v{VT}, v{O0 + 31}, %[gp] sc1")
            e("s_mov_b64 exec, s[%d:%d]" % (TA, TA + 1))
            if pub == "lds":
                e("s_sub_u32 %[x2], %[b], 1")
                e(f"v_mov_b32_e32 v{VT2}, %[x2]")
                e(f"ds_write_b32 %[anp], v{VT2}")
            e(f"L_nopub{k}_%=:")
        e(f"v_mov_b32_e32 v{VT2}, %[x1]")
        if not border:
            e(f"ds_write_b32 %[acn], v{VT2}")
        if trailing:
            e(f"ds_write_b32 %[atl], v{VT2}")
        e("s_mov_b32 %[b], %[x1]")

    # prologue: the first block's subject words into set 0
    e("s_add_u32 %[x1], %[b], 1")
    wait(e, "sfp", "%[sf]", "%[x1]", "%[asf]", "%[nsf]" if ts else None)
    e("s_and_b32 %[x2], %[b], 31")
    e("s_lshl_b32 %[x2], %[x2], 11")
    e(f"v_add_u32_e32 v{VA}, %[x2], %[skb]")
    for i in range(4):
        e(f"ds_read2st64_b32 v[{SK0 + 2 * i}:{SK0 + 2 * i + 1}], v{VA} offset0:{2 * i} offset1:{2 * i + 1}")
    e("L_top_%=:")
    body(0)
    e("s_cmp_lt_u32 %[b], %[be]")
    e("s_cbranch_scc0 L_done_%=")
    body(1)
    e("s_cmp_lt_u32 %[b], %[be]")
    e("s_cbranch_scc1 L_top_%=")
    e("L_done_%=:")
    e("s_mov_b32 %[st], 0")
    e("s_branch L_end_%=")
    e("L_timeout_%=:")
    e("s_mov_b32 %[st], 1")
    e("L_end_%=:")
    return out


# ------------------------------------------------------- affine, round 3 --
# Registers of gen_aff2 (TOP pairs / cell pairs as gen_loop_aff).
B_AW, B_AA, B_AT, B_AP = 136, 137, 138, 139   # cmp weight, diag + weight, temp, poll result
B_SK0, B_SK1 = 140, 148                          # subject words (codes), double buffered
B_VT, B_VT2, B_VA, B_VB = 156, 157, 158, 159    # temps / LDS addresses
B_WB = 160                                       # LUT weight bytes of 4 steps


NEG_INF = -(1 << 29)   # kAffNeg
# gen_aff2 step order (round 4): 1 = no VALU reads the previous instruction's result
REORDER = int(os.environ.get("ANYSEQ_GEN_REORDER", "1"))
# gen_aff2 LDS publish (round 4): 1 = the slot address once per block, counter inside the exec window
SLIM = int(os.environ.get("ANYSEQ_GEN_SLIM", "1"))
# gen_aff2 issue slots (round 5): a wave alone on its SIMD issues about one instruction
# per 4-5 cycles whatever its kind, so every SALU, s_waitcnt and LDS instruction of the
# block costs a step's worth of VALU slots.  1 = the lean block: loop-carried diagonal /
# top-row state in the rotation's own registers (no block-end moves), 4 counted LDS waits
# per block instead of 16, the ring-slot check every other block, 2b kept in an SGPR, the
# consumption counters every other block.  A/B (gpurun_out/r05d, one box): the loop alone
# 61.9 -> 58.1 cycles per step (X space, LDS publisher), configs[2] 517 -> 535 GCUPS.
# 2 = also the subject-prefetch wait every other block (r05f: configs[2] 544 -> 551 GCUPS).
LEAN = int(os.environ.get("ANYSEQ_GEN_LEAN", "2"))
# gen_aff2 subject codes (round 5): 1 = two 16-byte loads per lane and block from the
# problem's code rows in HBM (DPProblem::scode; kernel ANYSEQ_AFF_GS 1), issued one block
# ahead; 0 = the I/O wave's pre-skewed LDS copy (ds_read2st64 at step 8, an s_filled wait)
GS = int(os.environ.get("ANYSEQ_GEN_GS", "1"))
# gen_aff2 hand-off reads (round 6): 1 = a consumer band issues the producer's counter
# read and the half's top-row reads back to back and checks the counter afterwards (the
# LDS serves one wave's requests in order and the producer writes the data before the
# counter, so a satisfied counter read validates the data reads issued after it); a failed
# check falls back to the poll loop and reads again.  The first half at the block start
# (one LDS round trip instead of a poll round trip followed by the reads), the second half
# issued at SPEC_B_ISSUE and checked at SPEC_B_CHECK (0: the round-5 counter poll at step
# 10, checked at 14, then the reads).
SPEC = int(os.environ.get("ANYSEQ_GEN_SPEC", "1"))
# 2 = as 1, but the first half of block b+1 is read (counter + data) at step SPEC_A of
# block b (and at the loop's entry for its first block) and only checked at b+1's start:
# the counter's round trip leaves the block start when the producer is a few steps ahead
SPEC_A = int(os.environ.get("ANYSEQ_GEN_SPEC_A", "29"))
SPEC_B_ISSUE = int(os.environ.get("ANYSEQ_GEN_SPEC_BI", "14"))
SPEC_B_CHECK = int(os.environ.get("ANYSEQ_GEN_SPEC_BC", "16"))
# diagnostic build (ts variants): 1 = only the steady-state start / end stamps, no per-block
# event checks (a step close to the product's: band lags in product steps)
TSLIGHT = int(os.environ.get("ANYSEQ_GEN_TSLIGHT", "0"))
AT0, AO0 = 64, 128          # TOP (G,F) pairs v64..v127, cell (G,F) pairs v128..v135 (step u: u % 4)


BR0 = 162          # rows per lane > 1: row k >= 1's cell (G, F) pairs from v(BR0 + 10 (k-1)), then
                   # its diagonal + weight and LUT weight bytes (row 1: v162..v169, v170, v171)
ROWTAG = {0: "", 1: "b", 2: "x"}   # named operands of row k: %[e], %[eb], %[ex] ... (%[ec]: a capture)
B_WBB = BR0 + 9    # (two rows: the last clobbered register)


def OGk_(k, u):
    return OG_(u) if k == 0 else v(BR0 + 10 * (k - 1) + 2 * (u % 4))


def OFk_(k, u):
    return OF_(u) if k == 0 else v(BR0 + 10 * (k - 1) + 2 * (u % 4) + 1)


def OGB_(u):
    return OGk_(1, u)


def OFB_(u):
    return OFk_(1, u)


def gen_aff2(kind, border, pub, lut, ts=False, epi=False, cap=True, nrows=1, lin=False, pro=False):
    """Affine steady-state loop, round 3: full blocks b .. be-1.
    kind G: G space (X_G = X + (r+c+2)|ge|), no clamp, no best (amode 0).
    kind L: X space (X = H + (r+2)|ge|, a per-ROW shift): the local clamp H >= 0 is
            X >= zl, a per-lane constant, folded into the E update
            (E' = max3(E, X_left + go, zl - ge) + ge keeps E' = max(E, 0)), and the
            best cell is max X per lane (H = X - (r+2)|ge| after the loop): no
            per-step offset, no SALU in the step.
    lut: the diagonal weight of 4 steps from ONE v_perm_b32 of the lane's 8-entry
         weight table (query code against subject codes 0..7; code 0xFF -> -1)
         and a byte-select SDWA add; else v_cmp + v_cndmask (any codes).
    Hand-off in HALF chunks (16 columns; the ring counters count halves): lane 63's
    cells leave through a DPP wave_shl:1 shift register, whose lanes 48..63 hold the
    chunk's first 16 columns after step 16 and its last 16 at the block end -- one
    ds_write_b64 / global_store_dwordx2 per half.  The consumer reads the first half of
    its top row at the block start (waiting for half 2b) and the second half at step 14
    (half 2b+1, polled at step 10), so a band trails the one above by about 2.6 blocks
    (64 steps of skew + 16 of granularity + latency) instead of whole chunks.
    Subject codes of the next block at step 8.
    epi: the band's last blocks (some lanes past the last column w-1): every lane keeps
    computing past w (subject code 0xFF; those cells feed no real cell), polls stop at
    the last half (nch = 2 x chunks), the best takes real cells only, and each lane
    captures its state at column w-1 (per-lane countdown cnt) into gc / ec / fc.
    cap False (round 4, the AF2F variants): an epilogue for bands whose column-(w-1)
    state nobody reads (no out_col / out_col_e / last-row F / last-column best: the
    transposed Hirschberg halves and the score fronts): no capture, and the best over
    every cell as in the main loop -- a cell right of column w-1 (subject code 0xFF,
    weight -1) never exceeds some real cell (its diagonal, E and F terms are each below
    a real cell's H; the clamp's 0 is a real cell's floor too), so the maximum is the
    same.  The capture made the epilogue ~1.6x slower per step, and every band's
    epilogue sits on the band chain (a consumer's last main-loop block waits for its
    producer's last publish, at the producer's epilogue end).
    r2 (round 5): two rows per lane -- lane l holds rows 2l (A) and 2l+1 (B) of a 128-row
    band at the same column.  A's step is the one-row step with the lane shift reading
    B's cells of the lane above (%[cur] / %[fd] are B's); B follows without a lane
    shift: its diagonal is A's cell of the previous step (OG_(u-1); at step 0 the
    loop-carried %[ga]), its up and F-in A's new cell, its own E chain (%[eb] / %[hgb]),
    weights (%[qb] or %[llb] / %[lhb]), clamp bound (%[zlpb]) and best (%[bestb]).  The
    shift register, the publish and the block-end state carry B's cells (the band's bottom
    row), so the hand-off is the one-row kernel's.  The DPP moves are shared by two cells:
    16.4 instead of 2 x 11.2 instructions per step (tools/micro/gen_mix_micro.py).
    nrows 3: rows 3l, 3l+1, 3l+2 the same way (row k from row k-1; %[gb] carries row B's
    cell of the previous step into row C's diagonal; %[ex] / %[hgx] / ... row C's).
    lin (round 5): the LINEAR gap recurrence in the same loop (the affine one with gap open
    0, where E = the left cell and F = the cell above): G space G = max3(G_diag + w,
    G_left, G_up); X space (kind L, local) X = max3(X_diag + w, max(X_left, zl') - |ge|,
    X_up) with zl' = %[zlp] = the clamp bound + |ge|.  One DPP and one shift-register move
    per step; the published pairs carry (G, G) (F-down = G), and at loop exit %[fd], %[e]
    and %[hg] get the last cell (the C++ blocks' affine step with open 0 then continues
    exactly: E and F of the next cell are the left and upper cells).
    pro (round 5): the band's first blocks with a zero-open left border (semiglobal), which
    the virtual prologue cannot reproduce: the lane's cell at column -1 (after %[pcnt]
    steps) is forced to the border %[pbrd] right after its max3, before anything reads it."""
    L = kind == "L"
    r2 = nrows > 1
    assert not (lin and r2) and not (pro and (r2 or epi))

    def force(u):
        if pro:
            e("v_cmp_eq_u32_e32 vcc, 0, %[pcnt]")
            e(f"v_cndmask_b32_e32 {OG_(u)}, {OG_(u)}, %[pbrd], vcc")
            e("v_add_u32_e32 %[pcnt], -1, %[pcnt]")
    last = nrows - 1
    assert not r2 or (REORDER and LEAN and SLIM and GS and not ts)
    OGP, OFP = (lambda u: OGk_(last, u)), (lambda u: OFk_(last, u))   # the published / lane-shifted cells
    PUBREG = int(OGk_(last, 3)[1:])
    trailing = pub != "lds"
    out = []
    e = out.append
    sets = (B_SK0, B_SK1)

    def code_loads(breg, dst):
        """GS: the lane's 32 subject codes of block `breg` into v[dst .. dst+7]: row bytes
        %[skb] + 32 breg (two dword-aligned 16-byte loads from the code rows %[sg])."""
        e(f"s_lshl_b32 %[x2], {breg}, 5")
        e(f"v_add_u32_e32 v{B_VA}, %[x2], %[skb]")
        e(f"global_load_dwordx4 v[{dst}:{dst + 3}], v{B_VA}, %[sg]")
        e(f"global_load_dwordx4 v[{dst + 4}:{dst + 7}], v{B_VA}, %[sg] offset:16")

    # GS: VMEM operations a block issues after its code loads (the vmcnt a block waits
    # with for its own codes): the glob publisher's two half stores (the diagnostic
    # build's event stores only add younger operations: the wait then covers a few more)
    code_wait = 2 if pub == "glob" else 0

    def top_reads(half):
        """8 ds_read_b128 of top-row pairs [16*half, 16*half+16) (chunk address in VB)."""
        for i in range(8):
            reg = AT0 + 32 * half + 4 * i
            e(f"ds_read_b128 v[{reg}:{reg + 3}], v{B_VB} offset:{128 * half + 16 * i}")

    def ring_addr(breg):
        # ring byte address of chunk `breg` into VB: rb + ((breg << 8) & 4095)
        e(f"s_lshl_b32 %[x2], {breg}, 8")
        e("s_and_b32 %[x2], %[x2], 4095")
        e("s_add_u32 %[x2], %[x2], %[rb]")
        if epi and not cap:
            # blocks past the last chunk (2b >= nch; the polls stop at the last half):
            # the top row from the "minus infinity" area, not a ring slot nobody
            # published for them
            e(f"s_lshl_b32 %[x4], {breg}, 1")
            e("s_cmp_ge_u32 %[x4], %[nch]")
            e("s_cselect_b32 %[x2], %[neg], %[x2]")
        e(f"v_mov_b32_e32 v{B_VB}, %[x2]")

    def border_write(breg):
        # band 0: lanes write the top border (value, value + go) of columns 32*breg + lane
        e(f"s_lshl_b32 %[x0], {breg}, 5")
        e("s_mul_i32 %[x2], %[x0], %[bvs]")
        e(f"v_add_u32_e32 v{B_VT}, %[x2], %[bvb]")
        e(f"v_add_u32_e32 v{B_VT2}, %[go], v{B_VT}")
        e("s_lshl_b32 %[x2], %[x0], 3")
        e(f"v_add_u32_e32 v{B_VA}, %[x2], %[lid8]")
        e(f"v_and_b32_e32 v{B_VA}, 0xfff, v{B_VA}")
        e(f"v_add_u32_e32 v{B_VA}, %[rb], v{B_VA}")
        e(f"ds_write_b64 v{B_VA}, v[{B_VT}:{B_VT2}]")

    # lean (non-border variants, where x0 is free): 2b in x0, set at the block start
    b2 = LEAN and not border
    spec = SPEC and not border and (not ts or TSLIGHT) and LEAN
    assert not SPEC or (SPEC_B_ISSUE < SPEC_B_CHECK <= 16 and 18 <= SPEC_A <= 31)

    def spec_prefetch(breg):
        """SPEC 2: the counter, then the first half of block `breg`'s top row (VB)."""
        ring_addr(breg)
        e(f"ds_read_b32 v{B_AP}, %[apr]")
        top_reads(0)

    def spec_first2(k):
        """SPEC 2, block start: the prefetched counter covers half 2b (x4) -> the reads
        issued after it are valid; else poll and read again."""
        e("s_waitcnt lgkmcnt(8)")
        e(f"v_readfirstlane_b32 %[x2], v{B_AP}")
        e("s_max_u32 %[sp], %[sp], %[x2]")
        e("s_cmp_ge_u32 %[sp], %[x4]")
        e(f"s_cbranch_scc1 L_sad{k}_%=")
        wait(e, f"pa{k}", "%[sp]", "%[x4]", "%[apr]", tmp=B_VT2)
        top_reads(0)
        e(f"L_sad{k}_%=:")

    def spec_first(k):
        """First half of the block's top row (half 2b, target in x4): the cached counter
        suffices -> read; else counter + reads together, check, poll loop on a miss."""
        e("s_cmp_ge_u32 %[sp], %[x4]")
        e(f"s_cbranch_scc1 L_sar{k}_%=")
        e(f"ds_read_b32 v{B_AP}, %[apr]")
        top_reads(0)
        e("s_waitcnt lgkmcnt(8)")
        e(f"v_readfirstlane_b32 %[x2], v{B_AP}")
        e("s_max_u32 %[sp], %[sp], %[x2]")
        e("s_cmp_ge_u32 %[sp], %[x4]")
        e(f"s_cbranch_scc1 L_sad{k}_%=")
        wait(e, f"pa{k}", "%[sp]", "%[x4]", "%[apr]", tmp=B_VT2)
        e(f"L_sar{k}_%=:")
        top_reads(0)
        e(f"L_sad{k}_%=:")

    def spec_second_issue():
        e(f"ds_read_b32 v{B_AP}, %[apr]")
        top_reads(1)

    def spec_second_check(k):
        """Second half (2b+1, needed at step 17): the reads issued at SPEC_B_ISSUE after the
        counter read are valid if that counter read covers the half."""
        half_target(2)
        e("s_waitcnt lgkmcnt(8)")
        e(f"v_readfirstlane_b32 %[x2], v{B_AP}")
        e("s_max_u32 %[sp], %[sp], %[x2]")
        e("s_cmp_ge_u32 %[sp], %[x4]")
        e(f"s_cbranch_scc1 L_sbd{k}_%=")
        wait(e, f"pb{k}", "%[sp]", "%[x4]", "%[apr]", tmp=B_VT2)
        top_reads(1)
        e(f"L_sbd{k}_%=:")

    def half_target(add):
        # x4 = 2b + add (clamped to the last half in the epilogue)
        if b2:
            e(f"s_add_u32 %[x4], %[x0], {add}")
        else:
            e("s_lshl_b32 %[x4], %[b], 1")
            e(f"s_add_u32 %[x4], %[x4], {add}")
        if epi:
            e("s_min_u32 %[x4], %[x4], %[nch]")

    def pub_counter(half):
        # x2 = 2(b-2) + half + 1 halves published (0 while b < 2)
        if b2:
            e(f"s_sub_u32 %[x2], %[x0], {3 - half}")
        else:
            e("s_lshl_b32 %[x2], %[b], 1")
            e(f"s_sub_u32 %[x2], %[x2], {3 - half}")
        e("s_max_i32 %[x2], %[x2], 0")

    EVB = 1000   # diagnostic build: the block whose hand-off events are recorded

    def event(k, slot, bval):
        """Diagnostic build: at block `bval` (b + const), store s_memrealtime to
        dbp[slot] (vector store from v138:139; the record pointer is 0 when off)."""
        if not ts or TSLIGHT:
            return
        e(f"s_cmp_eq_u32 %[b], {bval}")
        e(f"s_cbranch_scc0 L_ev{slot}{k}_%=")
        e("s_cmp_lg_u64 %[dbp], 0")
        e(f"s_cbranch_scc0 L_ev{slot}{k}_%=")
        e(f"s_memrealtime s[{TB}:{TB + 1}]")
        e("s_waitcnt lgkmcnt(0)")
        e(f"v_mov_b32_e32 v138, s{TB}")
        e(f"v_mov_b32_e32 v139, s{TB + 1}")
        e(f"v_mov_b32_e32 v{B_VT2}, 0")
        e(f"global_store_dwordx2 v{B_VT2}, v[138:139], %[dbp] offset:{8 * slot}")
        e(f"L_ev{slot}{k}_%=:")

    def event_last(k, slot, add):
        """Diagnostic build, band-end variants: when 2b + add is the band's last half
        (nch), store s_memrealtime to dbp[slot] (consumer: the last half seen, add 2;
        producer: the last half published, add -2)."""
        if not (ts and epi) or TSLIGHT:
            return
        e("s_lshl_b32 %[x2], %[b], 1")
        e(f"s_add_u32 %[x2], %[x2], {add & 0xffffffff}")
        e("s_cmp_eq_u32 %[x2], %[nch]")
        e(f"s_cbranch_scc0 L_evl{slot}{k}_%=")
        e("s_cmp_lg_u64 %[dbp], 0")
        e(f"s_cbranch_scc0 L_evl{slot}{k}_%=")
        e(f"s_memrealtime s[{TB}:{TB + 1}]")
        e("s_waitcnt lgkmcnt(0)")
        e(f"v_mov_b32_e32 v138, s{TB}")
        e(f"v_mov_b32_e32 v139, s{TB + 1}")
        e(f"v_mov_b32_e32 v{B_VT2}, 0")
        e(f"global_store_dwordx2 v{B_VT2}, v[138:139], %[dbp] offset:{8 * slot}")
        e(f"L_evl{slot}{k}_%=:")

    def count_miss(k, tag):
        if ts and not TSLIGHT:   # diagnostic: hand-off waits (block start or step 14)
            e("s_cmp_ge_u32 %[sp], %[x4]")
            e(f"s_cbranch_scc1 L_nm{tag}{k}_%=")
            e("s_add_u32 %[nmiss], %[nmiss], 1")
            e(f"L_nm{tag}{k}_%=:")

    def publish(k, half, reg):
        """Lanes 48..63 of the (G, F) pair `reg` hold 16 columns of chunk b-2: half
        `half` of the next band's top row (LDS: always written -- a dummy slot and
        counter 0 while b < 2 -- so the counted lgkmcnt waits stay fixed).  Linear: the
        pair's F register gets the cell first (F-down = G)."""
        if lin:
            e(f"v_mov_b32_e32 v{reg + 1}, v{reg}")
        if pub == "lds" and SLIM:
            # round 4: the slot address once per block (half 1 reuses it through the
            # offset field), the counter written by the same 16 lanes inside the exec
            # window, exec restored to all lanes (the loop runs with every lane active)
            if half == 0:
                e("s_sub_u32 %[x2], %[b], 2")
                e("s_lshl_b32 %[x2], %[x2], 8")
                e("s_and_b32 %[x2], %[x2], 4095")
                e("s_add_u32 %[x2], %[x2], %[nb]")
                e(f"v_add_u32_e32 v{B_VT}, %[x2], %[lo]")
            pub_counter(half)
            e(f"v_mov_b32_e32 v{B_VT2}, %[x2]")
            e("s_mov_b64 exec, %[hm]")
            e(f"ds_write_b64 v{B_VT}, v[{reg}:{reg + 1}] offset:{128 * half}")
            e(f"ds_write_b32 %[anp], v{B_VT2}")
            e("s_mov_b64 exec, -1")
            return
        if pub == "glob":
            e("s_cmp_lt_u32 %[b], 2")
            e(f"s_cbranch_scc1 L_nopub{half}{k}_%=")
        e("s_sub_u32 %[x2], %[b], 2")
        e("s_lshl_b32 %[x2], %[x2], 8")
        if pub == "lds":
            e("s_and_b32 %[x2], %[x2], 4095")
            e("s_add_u32 %[x2], %[x2], %[nb]")
        e(f"v_add_u32_e32 v{B_VT}, %[x2], %[lo]")
        e("s_mov_b64 s[%d:%d], exec" % (TA, TA + 1))
        e("s_mov_b64 exec, %[hm]")
        if pub == "lds":
            e(f"ds_write_b64 v{B_VT}, v[{reg}:{reg + 1}] offset:{128 * half}")
        else:
            e(f"global_store_dwordx2 v{B_VT}, v[{reg}:{reg + 1}], %[gp] offset:{128 * half} sc1")
        e("s_mov_b64 exec, s[%d:%d]" % (TA, TA + 1))
        if pub == "lds":
            pub_counter(half)
            e(f"v_mov_b32_e32 v{B_VT2}, %[x2]")
            e(f"ds_write_b32 %[anp], v{B_VT2}")
        if pub == "glob":
            e(f"L_nopub{half}{k}_%=:")

    def body(k):
        cs, ns = sets[k], sets[1 - k]
        e("s_add_u32 %[x1], %[b], 1")
        if b2:
            e("s_lshl_b32 %[x0], %[b], 1")
        if border:
            throttle(e, k)            # band 0 paces the chain (%[thr] s_sleep-1 units per block)
        event(k, 0, EVB + 2)          # producer: block EVB+2 starts
        event(k, 3, EVB)              # consumer: block EVB starts
        # ---- first half of this block's top row (half 2b)
        if not border:
            if spec and SPEC < 2:
                ring_addr("%[b]")     # (before the target: the band-end variant's uses x4)
            half_target(1)
            count_miss(k, "a")
            if spec and SPEC >= 2:
                spec_first2(k)
            elif spec:
                spec_first(k)
            else:
                wait(e, f"pa{k}", "%[sp]", "%[x4]", "%[apr]", tmp=B_VT2)
        event(k, 4, EVB)              # consumer: first half of chunk EVB seen
        if not spec:
            ring_addr("%[b]")
            top_reads(0)
        if GS:
            # this block's codes (loaded one block ago), then the next block's.  The glob
            # publisher stores its halves from block 2 on: blocks 0..2 wait for all.
            if code_wait:
                e("s_cmp_lt_u32 %[b], 3")
                e(f"s_cbranch_scc1 L_cw0{k}_%=")
                e(f"s_waitcnt vmcnt({code_wait})")
                e(f"s_branch L_cwd{k}_%=")
                e(f"L_cw0{k}_%=:")
                e("s_waitcnt vmcnt(0)")
                e(f"L_cwd{k}_%=:")
            else:
                e("s_waitcnt vmcnt(0)")
            code_loads("%[x1]", ns)
        if ts:
            e("s_cmp_lg_u32 %[tsf], 0")
            e(f"s_cbranch_scc1 L_nots{k}_%=")
            e("s_memrealtime %[ts]")
            e("s_waitcnt lgkmcnt(0)")
            e("s_mov_b32 %[tsf], 1")
            e(f"L_nots{k}_%=:")
        if pub == "lds" and not LEAN:
            # the next band's ring slot of chunk b-2 is free once it consumed chunk b-17
            e("s_cmp_lt_u32 %[b], 17")
            e(f"s_cbranch_scc1 L_nobp{k}_%=")
            e("s_sub_u32 %[x4], %[b], 17")
            wait(e, f"bp{k}", "%[sc]", "%[x4]", "%[anc]", tmp=B_VT2)
            e(f"L_nobp{k}_%=:")
        elif pub == "lds" and k == 1:
            # lean: every other block, for this block and the next (chunks b-2 and b-1:
            # consumed through chunk b-16); the loop's first block is checked at entry
            e("s_sub_u32 %[x4], %[b], 16")
            wait(e, f"bp{k}", "%[sc]", "%[x4]", "%[anc]", tmp=B_VT2, signed=True)
        g, f, dg = "%[cur]", "%[fd]", "%[dg]"
        if LEAN:
            # the diagonal and lane 0's top values of step 0 stay in the rotation's own
            # registers from the previous block (TG_30, TG_31 / TF_31); without the
            # publishing shift register the cell pair of step 31 does too
            dg = TG_(30)
            if pub == "none":
                g, f = OGP(31), OFP(31)
        nsub = (0 if GS else 4) + (1 if border else 0)   # subject reads (+ the border write) at step 8
        for u in range(32):
            if u == 8 and GS:
                if border:
                    border_write("%[x1]")
            elif u == 8:
                # next block's subject codes (other register set) and, band 0, its border.
                # Issued in every block (after the last one they read a stale slot, unused):
                # the counted lgkmcnt waits assume they are in flight.
                if LEAN < 2:
                    e("s_cmp_ge_u32 %[x1], %[be]")
                    e(f"s_cbranch_scc1 L_nopf{k}_%=")
                    e("s_add_u32 %[x4], %[b], 2")
                    wait(e, f"sf{k}", "%[sf]", "%[x4]", "%[asf]", tmp=B_VT2)
                    e(f"L_nopf{k}_%=:")
                elif k == 1:
                    # lean: every other block, for this block's prefetch and the next's
                    # (skewed blocks through b+2; the loop's first prefetch at entry)
                    e("s_add_u32 %[x4], %[b], 3")
                    e("s_min_u32 %[x4], %[x4], %[be]")
                    wait(e, f"sf{k}", "%[sf]", "%[x4]", "%[asf]", tmp=B_VT2)
                e("s_and_b32 %[x2], %[x1], 31")
                e("s_lshl_b32 %[x2], %[x2], 11")
                e(f"v_add_u32_e32 v{B_VA}, %[x2], %[skb]")
                for i in range(4):
                    e(f"ds_read2st64_b32 v[{ns + 2 * i}:{ns + 2 * i + 1}], v{B_VA} offset0:{2 * i} offset1:{2 * i + 1}")
                if border:
                    border_write("%[x1]")
            if spec and SPEC >= 2 and u == SPEC_A:
                spec_prefetch("%[x1]")
            if spec and u == SPEC_B_ISSUE:
                spec_second_issue()
            if spec and u == SPEC_B_CHECK:
                spec_second_check(k)
            if u == 10 and not border and not spec:
                # poll the producer's counter for the second half (used at step 14)
                e(f"ds_read_b32 v{B_AP}, %[apr]")
            if u == 14 and not spec:
                e("s_waitcnt lgkmcnt(0)")
                if not border:
                    e(f"v_readfirstlane_b32 %[x2], v{B_AP}")
                    e("s_max_u32 %[sp], %[sp], %[x2]")
                    half_target(2)
                    count_miss(k, "b")
                    wait(e, f"pb{k}", "%[sp]", "%[x4]", "%[apr]", tmp=B_VT2)
                    event(k, 5, EVB)      # consumer: second half seen
                    event_last(k, 13, 2)  # consumer: the band's last half seen
                top_reads(1)
            if LEAN:
                # lean: reads 0-3 of the first half by step 1, 4-7 by step 9 (the subject
                # reads and band 0's border write of step 8 may be in flight), the second
                # half (issued at step 14, ~3 steps earlier) by step 17 (the half-0 publish
                # of step 16 may be in flight)
                if u == 1:
                    e("s_waitcnt lgkmcnt(4)")
                if u == 9:
                    e(f"s_waitcnt lgkmcnt({nsub})")
                if u == 17:
                    e(f"s_waitcnt lgkmcnt({2 if pub == 'lds' else 0})")
            elif u in (1, 3, 5, 7, 9, 11, 13):
                i = (u - 1) // 2                   # first-half read holding T(u-1)
                allowed = (7 - i) + (nsub if u > 8 else 0) + (1 if (u > 10 and not border) else 0)
                e(f"s_waitcnt lgkmcnt({min(15, allowed)})")
            elif u >= 17 and u % 2 == 1:
                i = (u - 17) // 2                  # second-half read holding T(u-1)
                allowed = (7 - i) + (2 if pub == "lds" else 0)
                e(f"s_waitcnt lgkmcnt({min(15, allowed)})")
            sw = v(cs + u // 4)
            if LEAN:
                tg, tf = TG_((u - 1) % 32), TF_((u - 1) % 32)
            else:
                tg = "%[tfg]" if u == 0 else TG_(u - 1)
                tf = "%[tff]" if u == 0 else TF_(u - 1)
            # Instruction order (round 4): no VALU reads the result of the instruction
            # right before it -- E's max3 first, the DPP moves between the E pair, the
            # shift-register moves between OG -> hg -> F-down, the best after hg.
            if lin:
                # linear step: weight, the cell above by DPP (2 wait states after the left
                # cell's max3: s_nop where the weight and the shift register leave fewer)
                sr = u >= 2 and pub != "none"
                # VALU since the left cell's max3: the previous step's shift-register move (the
                # block's first step follows the block start's moves, waits and reads)
                nv = 2 if u == 0 else (1 if u - 1 >= 2 and pub != "none" else 0)
                if lut:
                    if u % 4 == 0:
                        e(f"v_perm_b32 v{B_WB}, %[lh], %[ll], {sw}")
                        nv += 1
                    e(f"v_add_u32_sdwa v{B_AA}, {dg}, sext(v{B_WB}) dst_sel:DWORD dst_unused:UNUSED_PAD "
                      f"src0_sel:DWORD src1_sel:BYTE_{u % 4}")
                    nv += 1
                else:
                    e(f"v_cmp_eq_u32_sdwa vcc, %[q], {sw} src0_sel:DWORD src1_sel:BYTE_{u % 4}")
                    e(f"v_cndmask_b32_e32 v{B_AW}, %[wx], %[wm], vcc")
                    e(f"v_add_u32_e32 v{B_AA}, {dg}, v{B_AW}")
                    nv += 3
                if L:
                    e(f"v_max_i32_e32 v{B_AT}, {g}, %[zlp]")
                    e(f"v_add_u32_e32 v{B_AT}, %[ge], v{B_AT}")
                    nv += 2
                if nv < 2:
                    e(f"s_nop {1 - nv}")
                e(f"v_mov_b32_dpp {tg}, {g} wave_shr:1 row_mask:0xf bank_mask:0xf")
                e(f"v_max3_i32 {OG_(u)}, v{B_AA}, {'v' + str(B_AT) if L else g}, {tg}")
                force(u)
                if L and u % 2 == 1 and not (epi and cap):
                    e(f"v_max3_i32 %[best], %[best], {OG_(u - 1)}, {OG_(u)}")
                if sr:
                    e(f"v_mov_b32_dpp {OG_(u - 1)}, {OG_(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
            elif REORDER:
                if L:
                    e("v_max3_i32 %[e], %[e], %[hg], %[zlp]")
                else:
                    e("v_max_i32_e32 %[e], %[e], %[hg]")
            if lin:
                pass
            elif lut:
                if u % 4 == 0:
                    e(f"v_perm_b32 v{B_WB}, %[lh], %[ll], {sw}")
                e(f"v_add_u32_sdwa v{B_AA}, {dg}, sext(v{B_WB}) dst_sel:DWORD dst_unused:UNUSED_PAD "
                  f"src0_sel:DWORD src1_sel:BYTE_{u % 4}")
            else:
                e(f"v_cmp_eq_u32_sdwa vcc, %[q], {sw} src0_sel:DWORD src1_sel:BYTE_{u % 4}")
                e(f"v_cndmask_b32_e32 v{B_AW}, %[wx], %[wm], vcc")
                e(f"v_add_u32_e32 v{B_AA}, {dg}, v{B_AW}")
            sr = u >= 2 and pub != "none"
            if lin:
                pass
            elif REORDER:
                e(f"v_mov_b32_dpp {tf}, {f} wave_shr:1 row_mask:0xf bank_mask:0xf")
                if L:
                    e("v_add_u32_e32 %[e], %[ge], %[e]")
                e(f"v_mov_b32_dpp {tg}, {g} wave_shr:1 row_mask:0xf bank_mask:0xf")
                e(f"v_max3_i32 {OG_(u)}, v{B_AA}, %[e], {tf}")
                force(u)
                if sr and not r2:
                    e(f"v_mov_b32_dpp {OF_(u - 1)}, {OF_(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
                e(f"v_add_u32_e32 %[hg], %[go], {OG_(u)}")
                if L and u % 2 == 1 and not (epi and cap):
                    e(f"v_max3_i32 %[best], %[best], {OG_(u - 1)}, {OG_(u)}")
                if sr and not r2:
                    e(f"v_mov_b32_dpp {OG_(u - 1)}, {OG_(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
                e(f"v_max_i32_e32 {OF_(u)}, {tf}, %[hg]")
                for rk in range(1, nrows):
                    # row k: diagonal row k-1's previous cell, up / F-in its new cell, no lane shift
                    t = ROWTAG[rk]
                    dgk = OGk_(rk - 1, u - 1)   # (step 0: the rotation's last slot, loaded from %[ga] / %[gb])
                    aak, wbk = BR0 + 10 * (rk - 1) + 8, BR0 + 10 * (rk - 1) + 9
                    if L:
                        e(f"v_max3_i32 %[e{t}], %[e{t}], %[hg{t}], %[zlp{t}]")
                    else:
                        e(f"v_max_i32_e32 %[e{t}], %[e{t}], %[hg{t}]")
                    if lut:
                        if u % 4 == 0:
                            e(f"v_perm_b32 v{wbk}, %[lh{t}], %[ll{t}], {sw}")
                        e(f"v_add_u32_sdwa v{aak}, {dgk}, sext(v{wbk}) dst_sel:DWORD dst_unused:UNUSED_PAD "
                          f"src0_sel:DWORD src1_sel:BYTE_{u % 4}")
                    else:
                        e(f"v_cmp_eq_u32_sdwa vcc, %[q{t}], {sw} src0_sel:DWORD src1_sel:BYTE_{u % 4}")
                        e(f"v_cndmask_b32_e32 v{B_AW}, %[wx], %[wm], vcc")
                        e(f"v_add_u32_e32 v{aak}, {dgk}, v{B_AW}")
                    if L:
                        e(f"v_add_u32_e32 %[e{t}], %[ge], %[e{t}]")
                    e(f"v_max3_i32 {OGk_(rk, u)}, v{aak}, %[e{t}], {OFk_(rk - 1, u)}")
                    e(f"v_add_u32_e32 %[hg{t}], %[go], {OGk_(rk, u)}")
                    if L and u % 2 == 1 and not (epi and cap):
                        e(f"v_max3_i32 %[best{t}], %[best{t}], {OGk_(rk, u - 1)}, {OGk_(rk, u)}")
                    e(f"v_max_i32_e32 {OFk_(rk, u)}, {OFk_(rk - 1, u)}, %[hg{t}]")
                    if sr and rk == last:
                        e(f"v_mov_b32_dpp {OGk_(rk, u - 1)}, {OGk_(rk, u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
                        e(f"v_mov_b32_dpp {OFk_(rk, u - 1)}, {OFk_(rk, u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
            else:
                if L:
                    e("v_max3_i32 %[e], %[e], %[hg], %[zlp]")
                    e("v_add_u32_e32 %[e], %[ge], %[e]")
                else:
                    e("v_max_i32_e32 %[e], %[e], %[hg]")
                e(f"v_mov_b32_dpp {tf}, {f} wave_shr:1 row_mask:0xf bank_mask:0xf")
                e(f"v_mov_b32_dpp {tg}, {g} wave_shr:1 row_mask:0xf bank_mask:0xf")
                e(f"v_max3_i32 {OG_(u)}, v{B_AA}, %[e], {tf}")
                e(f"v_add_u32_e32 %[hg], %[go], {OG_(u)}")
                e(f"v_max_i32_e32 {OF_(u)}, {tf}, %[hg]")
            if epi and cap:
                if L:
                    # best over real cells only (cnt >= 0: column <= w-1)
                    e(f"v_max_i32_e32 v{B_AT}, %[best], {OG_(u)}")
                    e("v_cmp_le_i32_e32 vcc, 0, %[cnt]")
                    e(f"v_cndmask_b32_e32 %[best], %[best], v{B_AT}, vcc")
                    for rk in range(1, nrows):
                        t = ROWTAG[rk]
                        e(f"v_max_i32_e32 v{B_AT}, %[best{t}], {OGk_(rk, u)}")
                        e(f"v_cndmask_b32_e32 %[best{t}], %[best{t}], v{B_AT}, vcc")
                # the lane whose cell is column w-1 at this step keeps its state
                e("v_cmp_eq_u32_e32 vcc, 0, %[cnt]")
                e(f"v_cndmask_b32_e32 %[gc], %[gc], {OG_(u)}, vcc")
                if lin:
                    # (linear: F-down = the cell; E = the left cell, G space -- the kernel
                    # never asks a linear band for out_col_e)
                    e(f"v_cndmask_b32_e32 %[ec], %[ec], {g}, vcc")
                    e(f"v_cndmask_b32_e32 %[fc], %[fc], {OG_(u)}, vcc")
                else:
                    e("v_cndmask_b32_e32 %[ec], %[ec], %[e], vcc")
                if lin:
                    pass
                elif r2:
                    # (a row's F-down is the next row's F-in: only the last row's is kept)
                    for rk in range(1, nrows):
                        t = ROWTAG[rk]
                        e(f"v_cndmask_b32_e32 %[gc{t}], %[gc{t}], {OGk_(rk, u)}, vcc")
                        e(f"v_cndmask_b32_e32 %[ec{t}], %[ec{t}], %[e{t}], vcc")
                    e(f"v_cndmask_b32_e32 %[fc], %[fc], {OFk_(last, u)}, vcc")
                else:
                    e(f"v_cndmask_b32_e32 %[fc], %[fc], {OF_(u)}, vcc")
                e("v_add_u32_e32 %[cnt], -1, %[cnt]")
            if not REORDER:
                if L and u % 2 == 1 and not (epi and cap):
                    e(f"v_max3_i32 %[best], %[best], {OG_(u - 1)}, {OG_(u)}")
                if sr:
                    e(f"v_mov_b32_dpp {OG_(u - 1)}, {OG_(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
                    e(f"v_mov_b32_dpp {OF_(u - 1)}, {OF_(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
            if u == 16 and pub != "none":
                publish(k, 0, PUBREG)              # cell pair of step 15: steps 0..15 in lanes 48..63
                event(k, 1, EVB + 2)               # producer: first half of chunk EVB published
            g, f, dg = OGP(u), OFP(u), tg
        if not LEAN or pub != "none":
            e(f"v_mov_b32_e32 %[cur], {OGP(31)}")
            # (linear: F-down = the cell; also the shift move's second wait state)
            e(f"v_mov_b32_e32 %[fd], {OGP(31) if lin else OFP(31)}")
        if not LEAN:
            e(f"v_mov_b32_e32 %[dg], {TG_(30)}")
        if pub != "none":
            e(f"v_mov_b32_dpp {OGP(31)}, {OGP(30)} wave_shl:1 row_mask:0xf bank_mask:0xf")
            if not lin:
                e(f"v_mov_b32_dpp {OFP(31)}, {OFP(30)} wave_shl:1 row_mask:0xf bank_mask:0xf")
        if not LEAN:
            e(f"v_mov_b32_e32 %[tfg], {TG_(31)}")
            e(f"v_mov_b32_e32 %[tff], {TF_(31)}")
        if pub != "none":
            publish(k, 1, PUBREG)                  # pair of step 31: steps 16..31 in lanes 48..63
            event(k, 2, EVB + 2)                   # producer: second half published
            event_last(k, 14, -2)                  # producer: the band's last half published
        event(k, 6, EVB)                           # consumer: block EVB ends
        if not LEAN or k == 1:
            # (lean: every other block -- a consumption counter one block behind only
            # holds the producer and the I/O wave one ring slot further back)
            e(f"v_mov_b32_e32 v{B_VT2}, %[x1]")
            if not border:
                e(f"ds_write_b32 %[acn], v{B_VT2}")
            if trailing:
                e(f"ds_write_b32 %[atl], v{B_VT2}")
        e("s_mov_b32 %[b], %[x1]")

    # the first block's subject codes into set 0 (band 0: and its border)
    e("s_add_u32 %[x1], %[b], 1")
    if GS:
        code_loads("%[b]", B_SK0)
    else:
        wait(e, "sfp", "%[sf]", "%[x1]", "%[asf]", tmp=B_VT2)
        e("s_and_b32 %[x2], %[b], 31")
        e("s_lshl_b32 %[x2], %[x2], 11")
        e(f"v_add_u32_e32 v{B_VA}, %[x2], %[skb]")
        for i in range(4):
            e(f"ds_read2st64_b32 v[{B_SK0 + 2 * i}:{B_SK0 + 2 * i + 1}], v{B_VA} offset0:{2 * i} offset1:{2 * i + 1}")
    if border:
        border_write("%[b]")
    e("s_waitcnt lgkmcnt(0)")
    if GS:
        e("s_waitcnt vmcnt(0)")
    # lean: the loop-carried diagonal / top values (and without publishing, the cell
    # pair) live in the rotation's registers; the ring slot of the first block's
    # publish is checked here (the loop checks every other block)
    lean_regs = [("%[dg]", TG_(30)), ("%[tfg]", TG_(31)), ("%[tff]", TF_(31))]
    if pub == "none":
        lean_regs += [("%[cur]", OGP(31)), ("%[fd]", OFP(31))]
    for k in range(nrows - 1):
        # row k's cell of the previous step: row k+1's diagonal at step 0
        lean_regs += [("%[g" + "ab"[k] + "]", OGk_(k, 31))]
    if LEAN:
        for named, reg in lean_regs:
            e(f"v_mov_b32_e32 {reg}, {named}")
        if LEAN >= 2 and not GS:
            e("s_add_u32 %[x4], %[b], 2")
            e("s_min_u32 %[x4], %[x4], %[be]")
            wait(e, "sfe", "%[sf]", "%[x4]", "%[asf]", tmp=B_VT2)
        if pub == "lds":
            e("s_sub_u32 %[x4], %[b], 17")
            wait(e, "bpe", "%[sc]", "%[x4]", "%[anc]", tmp=B_VT2, signed=True)
    if SPEC >= 2 and not border and (not ts or TSLIGHT) and LEAN:
        spec_prefetch("%[b]")     # (the loop's first block)
    e("L_top_%=:")
    body(0)
    e("s_cmp_lt_u32 %[b], %[be]")
    e("s_cbranch_scc0 L_done_%=")
    body(1)
    e("s_cmp_lt_u32 %[b], %[be]")
    e("s_cbranch_scc1 L_top_%=")
    e("L_done_%=:")
    e("s_waitcnt lgkmcnt(0)")
    if ts:
        e("s_memrealtime %[te]")
        e("s_waitcnt lgkmcnt(0)")
    e("s_mov_b32 %[st], 0")
    e("s_branch L_end_%=")
    e("L_timeout_%=:")
    e("s_waitcnt lgkmcnt(0)")
    e("s_mov_b32 %[st], 1")
    e("L_end_%=:")
    if LEAN:
        for named, reg in lean_regs:
            e(f"v_mov_b32_e32 {named}, {reg}")
    if lin:
        # the C++ blocks' open-0 affine step: F-down, E and G + go of the last cell
        for named in ("%[fd]", "%[e]", "%[hg]"):
            e(f"v_mov_b32_e32 {named}, %[cur]")
    return out


def TG_(u):
    return v(AT0 + 2 * u)


def TF_(u):
    return v(AT0 + 2 * u + 1)


def OG_(u):
    # step u's cell pair: four pairs in rotation -- a cell is read by the next step
    # (DPP source, best) and then holds the publishing shift register for one step
    return v(AO0 + 2 * (u % 4))


def OF_(u):
    return v(AO0 + 2 * (u % 4) + 1)


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    dst = os.path.join(here, "..", "anyseq_amd", "csrc", "anyseq_block_asm.inc")
    if len(sys.argv) > 1:   # (experimental builds: another file, e.g. ANYSEQ_GEN_LEAN=1)
        dst = sys.argv[1]
    lines = ["// GENERATED by tools/gen_block_asm.py -- do not edit.", ""]
    variants = [("G", "G", {}), ("L", "L", {}),
                # timing variants for tools/micro/block_micro.hip
                ("G_NOST", "G", {"stores": False}), ("G_NORD", "G", {"reads": False}),
                ("G_NONE", "G", {"stores": False, "reads": False}),
                ("G_ALLST", "G", {"reads": False, "store_mode": "all"}),
                ("G_EXONLY", "G", {"reads": False, "store_mode": "exec_only"}),
                ("G_EXEC", "G", {"store_mode": "exec"})]
    for name, kind, kw in variants:
        body = gen(kind, **kw)
        lines.append(f"#define ANYSEQ_BLOCK_ASM_{name} \\")
        for ln in body:
            lines.append(f'    "{ln}\\n" \\')
        lines.append("")
    for kind in ("G", "L"):
        for border in (0, 1):
            for pub in ("none", "lds", "glob"):
                for ts in (False, True):
                    name = f"ANYSEQ_LOOP2_{kind}_B{border}_{pub.upper()}" + ("_TS" if ts else "")
                    lines.append(f"#define {name} \\")
                    for ln in gen_loop2(kind, border, pub, ts):
                        lines.append(f'    "{ln}\\n" \\')
                    lines.append("")
    for kind in ("G", "L"):
        for border in (0, 1):
            for pub in ("none", "lds", "glob"):
                for lut in (0, 1):
                    for ts in (False, True):
                        for epi, cap, tag in ((False, True, ""), (True, True, "E"), (True, False, "F")):
                            name = (f"ANYSEQ_AF2{tag}_{kind}_B{border}_{pub.upper()}_U{lut}"
                                    + ("_TS" if ts else ""))
                            lines.append(f"#define {name} \\")
                            for ln in gen_aff2(kind, border, pub, lut, ts, epi, cap):
                                lines.append(f'    "{ln}\\n" \\')
                            lines.append("")
    # zero-open left border prologue (one row per lane, affine G / L and linear N / M kinds)
    for kind, lk, lin in (("G", "G", False), ("L", "L", False), ("G", "N", True), ("L", "M", True)):
        for border in (0, 1):
            for pub in ("none", "lds", "glob"):
                for lut in (0, 1):
                    name = f"ANYSEQ_AF2P_{lk}_B{border}_{pub.upper()}_U{lut}"
                    lines.append(f"#define {name} \\")
                    for ln in gen_aff2(kind, border, pub, lut, False, False, True, lin=lin, pro=True):
                        lines.append(f'    "{ln}\\n" \\')
                    lines.append("")
    # linear gap in the affine loop (one row per lane, no diagnostic-stamp variants):
    # kinds N (G space) and M (X space: local)
    for kind, lk in (("G", "N"), ("L", "M")):
        for border in (0, 1):
            for pub in ("none", "lds", "glob"):
                for lut in (0, 1):
                    for epi, cap, tag in ((False, True, ""), (True, True, "E"), (True, False, "F")):
                        name = f"ANYSEQ_AF2{tag}_{lk}_B{border}_{pub.upper()}_U{lut}"
                        lines.append(f"#define {name} \\")
                        for ln in gen_aff2(kind, border, pub, lut, False, epi, cap, lin=True):
                            lines.append(f'    "{ln}\\n" \\')
                        lines.append("")
    # two and three rows per lane (no diagnostic-stamp variants)
    for nrows, pre in ((2, "AF2R"), (3, "AF2R3")):
        for kind in ("G", "L"):
            for border in (0, 1):
                for pub in ("none", "lds", "glob"):
                    for lut in (0, 1):
                        for epi, cap, tag in ((False, True, ""), (True, True, "E"), (True, False, "F")):
                            name = f"ANYSEQ_{pre}{tag}_{kind}_B{border}_{pub.upper()}_U{lut}"
                            lines.append(f"#define {name} \\")
                            for ln in gen_aff2(kind, border, pub, lut, False, epi, cap, nrows=nrows):
                                lines.append(f'    "{ln}\\n" \\')
                            lines.append("")
    sclob = ", ".join(f'"s{n}"' for n in range(TA, TB + 2))
    clob = ", ".join(f'"v{n}"' for n in range(AT0, B_WB + 1))
    lines.append(f"#define ANYSEQ_AF2_ASM_CLOBBERS {clob}, {sclob}, \"vcc\", \"scc\"")
    clob = ", ".join(f'"v{n}"' for n in range(AT0, B_WBB + 1))
    lines.append(f"#define ANYSEQ_AF2R_ASM_CLOBBERS {clob}, {sclob}, \"vcc\", \"scc\"")
    clob = ", ".join(f'"v{n}"' for n in range(AT0, BR0 + 20))
    lines.append(f"#define ANYSEQ_AF2R3_ASM_CLOBBERS {clob}, {sclob}, \"vcc\", \"scc\"")
    clob = ", ".join(f'"v{n}"' for n in range(T0, A + 1))
    lines.append(f"#define ANYSEQ_BLOCK_ASM_CLOBBERS {clob}, \"vcc\"")
    clob = ", ".join(f'"v{n}"' for n in range(T0, SKB_ + 8))
    sclob = ", ".join(f'"s{n}"' for n in range(TA, TB + 2))
    lines.append(f"#define ANYSEQ_LOOP2_ASM_CLOBBERS {clob}, {sclob}, \"vcc\", \"scc\"")

    lines.append("")
    with open(dst, "w") as f:
        f.write("\n".join(lines))
    print("wrote", dst)


if __name__ == "__main__":
    main()
