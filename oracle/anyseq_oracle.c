/*
 * anyseq_oracle.c — CPU restatement of the AnySeq reference CPU path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path (anyseq_amd/).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product library never links
 * or calls it.
 *
 * What it restates (reference files under /root/reference/src, read as text):
 *   - the per-cell recurrence          align.impala:46-79   (relax_global / relax_local)
 *   - borders / init                   align.impala:85-90
 *   - the linear scoring scheme        align.impala:130-150 (+2 / -1 / -1 in the ABI)
 *   - the linear-memory fill           iteration_cpu.impala:15-57, scoring_cpu.impala:1-85,
 *                                      scoring.impala:29-137,218-259
 *   - the column-split Hirschberg      align.impala:237-311, traceback_lintime.impala:1-148,
 *                                      iteration_cpu.impala:59-173, scoring.impala:261-328,
 *                                      scoring_cpu.impala:87-157
 *   - blockwise predecessors           predecessors.impala:36-61, mapping_cpu.impala:67-84
 *   - the traceback walk / out layout  traceback.impala:1-80
 *   - reduce_max / next_pow_2          utils.impala:12-49, iteration_cpu.impala:205-250
 * with `benchmark` restored to run its body once (utils.impala:164-189; see
 * SURVEY.md §0.1), CPU BLOCK_WIDTH = BLOCK_HEIGHT = 1024 (iteration_cpu.impala:1-2),
 * and get_thread_count() = 4 by default (backend/backend_cpu.impala:13).
 *
 * Parity pinning: the reference toolchain (AnyDSL/Impala) is absent, so this
 * restatement is pinned by (1) the hand-derived known answers of SURVEY.md
 * Appendix C, (2) an independent textbook full-matrix DP (tests/), and (3)
 * committed golden fixtures generated from it (tests/golden/).
 *
 * Build-defined extension (no reference semantics, SURVEY.md §0.4/§8c —
 * "parity unpinned" by the reference): affine-gap (Gotoh) scores, see
 * oracle_affine_score() below; pinned by the reduction open == 0 => linear.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>

typedef int32_t Score;
typedef int32_t Index;
typedef uint8_t Pred;

#define SCORE_MIN_VALUE (-2147483647)      /* align.impala:16 */
#define MIN_PART_WIDTH_HB 128              /* align.impala:18 */
#define CPU_BW 1024                        /* iteration_cpu.impala:1 */
#define CPU_BH 1024                        /* iteration_cpu.impala:2 */
#define SPLIT_UNSET ((Score)0x7fff0000)    /* sentinel: split never written */

enum { PRED_NONE = 0, PRED_GAP_Q = 1, PRED_GAP_S = 2, PRED_NO_GAP = 3 };  /* align.impala:37-40 */
enum { SCHEME_GLOBAL = 0, SCHEME_SEMIGLOBAL = 1, SCHEME_LOCAL = 2 };

typedef struct {
    int kind;
    Score match, mismatch, gap;
} Scheme;

static int g_threads = 4;                   /* backend_cpu.impala:13 */
static int g_error = 0;                     /* set when an unset split is read */

void oracle_set_threads(int t) { g_threads = t < 1 ? 1 : t; }
int oracle_get_threads(void) { return g_threads; }
int oracle_last_error(void) { return g_error; }

/* ---------------------------------------------------------------- utils -- */
static inline Index imin(Index a, Index b) { return a < b ? a : b; }
static inline Index imax(Index a, Index b) { return a > b ? a : b; }
static inline Index imin3(Index a, Index b, Index c) { return imin(imin(a, b), c); }
static inline Index round_up_div(Index a, Index b) { return (a + b - 1) / b; }   /* utils.impala:12 */

static Index next_pow_2(Index i) {                                                 /* utils.impala:19 */
    if (i == 0) return 0;
    Index n = i - 1, r = 1;
    while (n > 0) { n >>= 1; r <<= 1; }
    return r;
}

/* Vector with logical index -1 at storage 0 (dynprog.impala:194-199). */
typedef struct { Score* buf; Index length; } Vec;
static Vec vec_create(Index length) {
    Vec v; v.length = length;
    Index mem = length + 1; if (mem < 1) mem = 1;
    v.buf = (Score*)calloc((size_t)mem, sizeof(Score));
    return v;
}
#define V(v, i) ((v).buf[(i) + 1])

/* ------------------------------------------------------ parallel-for ---- */
typedef void (*body_fn)(void* ctx, Index i);
typedef struct { body_fn fn; void* ctx; Index lo, hi; } par_arg;
static void* par_worker(void* p) {
    par_arg* a = (par_arg*)p;
    for (Index i = a->lo; i < a->hi; ++i) a->fn(a->ctx, i);
    return NULL;
}
/* AnyDSL `parallel(T, lo, hi)`: iterations are independent; static split. */
static void parallel_for(Index lo, Index hi, body_fn fn, void* ctx) {
    Index n = hi - lo;
    if (n <= 0) return;
    int T = g_threads;
    if (T <= 1 || n == 1) { for (Index i = lo; i < hi; ++i) fn(ctx, i); return; }
    if (T > n) T = n;
    pthread_t th[256]; par_arg args[256];
    if (T > 256) T = 256;
    Index chunk = (n + T - 1) / T;
    int used = 0;
    for (int t = 0; t < T; ++t) {
        Index a = lo + t * chunk, b = imin(hi, a + chunk);
        if (a >= b) break;
        args[t].fn = fn; args[t].ctx = ctx; args[t].lo = a; args[t].hi = b;
        pthread_create(&th[t], NULL, par_worker, &args[t]);
        ++used;
    }
    for (int t = 0; t < used; ++t) pthread_join(th[t], NULL);
}

/* --------------------------------------------------------- recurrence -- */
static inline Score init_scores(const Scheme* sc, Index i) {                   /* align.impala:85-86 */
    return sc->kind == SCHEME_GLOBAL ? (i + 1) * sc->gap : 0;
}
static inline Pred init_predc_rows(const Scheme* sc, Index i) {                /* align.impala:88,90 */
    if (sc->kind != SCHEME_GLOBAL) return PRED_NONE;
    return i == -1 ? PRED_NONE : PRED_GAP_S;
}
static inline Pred init_predc_cols(const Scheme* sc, Index i) {                /* align.impala:89,90 */
    if (sc->kind != SCHEME_GLOBAL) return PRED_NONE;
    return i == -1 ? PRED_NONE : PRED_GAP_Q;
}

/* relax_global / relax_local (align.impala:46-79); semiglobal uses global relax. */
static inline Score relax(const Scheme* sc, uint8_t q, uint8_t s,
                          Score ng, Score gq, Score gs, Pred* p) {
    Score score = ng + (q == s ? sc->match : sc->mismatch);
    Pred pr = PRED_NO_GAP;
    Score qgap = gq + sc->gap;
    if (qgap > score) { score = qgap; pr = PRED_GAP_Q; }
    Score sgap = gs + sc->gap;
    if (sgap > score) { score = sgap; pr = PRED_GAP_S; }
    if (sc->kind == SCHEME_LOCAL && 0 > score) { score = 0; pr = PRED_NONE; }
    *p = pr;
    return score;
}

/* Sequence accessor: forward read(i) = base[off + i], reversed base[off - i]
 * (dynprog.impala:536-548). */
typedef struct { const uint8_t* base; Index off; int rev; } SeqAcc;
static inline uint8_t seq_read(const SeqAcc* a, Index i) {
    return a->rev ? a->base[a->off - i] : a->base[a->off + i];
}

/* ----------------------------------------------- reduce_max (64 chunks) -- */
/* iteration_cpu.impala:205-250 + utils.impala:30-49: strict '>' => first index of max */
static void reduce_max(const Vec* v, Index offset, Index length, Score* out_score, Index* out_index) {
    const Index num_blocks = 64;
    Index block_size = round_up_div(length, num_blocks);
    Score pres[64]; Index pind[64];
    for (Index b = 0; b < num_blocks; ++b) {
        Index offs = offset + b * block_size;
        Index len = imin(block_size, length - b * block_size);
        Score score = SCORE_MIN_VALUE; Index index = -1;
        for (Index i = offs; i < offs + len; ++i) {
            Score x = V(*v, i);
            if (x > score) { score = x; index = i; }
        }
        pres[b] = score; pind[b] = index;
    }
    Score score = pres[0]; Index index = pind[0];
    for (Index i = 1; i < num_blocks; ++i)
        if (pres[i] > score) { score = pres[i]; index = pind[i]; }
    *out_score = score; *out_index = index;
}

/* ------------------------------------------------ linear-memory tiles ---- */
/* Local max tracking per slot (scoring_cpu.impala:37-85). */
typedef struct { Vec max_scores, max_i, max_j; } LocalMax;

/* One tile in the rolling linear-memory scheme (scoring_cpu.impala:1-35 for
 * linmem, :87-123 for the Hirschberg halves): `col` is the shared seam column
 * (logical index offset_i + i), `row` the shared row (offset_j + j), `corner`
 * the tile-column corner slot. */
typedef struct {
    const Scheme* sc;
    SeqAcc qa, sa;
    Vec* col; Index offset_i;
    Vec* row; Index offset_j;
    Score* corner;
    Index height, width;
    LocalMax* lm; Index slot;          /* local scheme only */
} LinTile;

static void lin_tile(LinTile* t) {
    const Scheme* sc = t->sc;
    Vec* col = t->col; Vec* row = t->row;
    const Index oi = t->offset_i, oj = t->offset_j, h = t->height, w = t->width;
    /* accessor prologue (scoring_cpu.impala:8-12): runs even for h <= 0 */
    Score no_gap = *t->corner;
    Score gap_q = 0;
    *t->corner = V(*col, oi + h - 1);
    Score blk_max = SCORE_MIN_VALUE; Index bmi = 0, bmj = 0;
    for (Index i = 0; i < h; ++i) {
        gap_q = V(*col, oi + i);                                   /* update_begin_line */
        uint8_t qs = seq_read(&t->qa, i);
        for (Index j = 0; j < w; ++j) {
            Pred p;
            Score s = relax(sc, qs, seq_read(&t->sa, j), no_gap, gap_q, V(*row, oj + j), &p);
            no_gap = V(*row, oj + j);                              /* write */
            gap_q = s;
            V(*row, oj + j) = s;
            if (t->lm && s > blk_max) { blk_max = s; bmi = i; bmj = j; }
        }
        no_gap = V(*col, oi + i);                                  /* update_end_line */
        V(*col, oi + i) = V(*row, oj + w - 1);
    }
    if (t->lm) {                                                   /* block_end */
        Index idx = t->slot;
        if (blk_max > V(t->lm->max_scores, idx)) {
            V(t->lm->max_scores, idx) = blk_max;
            V(t->lm->max_i, idx) = bmi + oi;
            V(t->lm->max_j, idx) = bmj + oj;
        }
    }
}

/* iteration (iteration_cpu.impala:15-57) over the linmem storage (scoring.impala:218-259). */
typedef struct {
    const Scheme* sc; const uint8_t* Q; const uint8_t* S; Index n, m;
    Vec *column, *row, *corners; LocalMax* lm;
    Index nbi, nbj, d;
} IterCtx;

static void iter_body(void* p, Index bdj) {
    IterCtx* c = (IterCtx*)p;
    Index bi = imin(c->d, c->nbi - 1) - bdj;
    Index bj = imax(c->d - c->nbi + 1, 0) + bdj;
    Index oi = bi * CPU_BH, oj = bj * CPU_BW;
    LinTile t;
    t.sc = c->sc;
    t.qa.base = c->Q; t.qa.off = oi; t.qa.rev = 0;
    t.sa.base = c->S; t.sa.off = oj; t.sa.rev = 0;
    t.col = c->column; t.offset_i = oi;
    t.row = c->row; t.offset_j = oj;
    t.corner = &V(*c->corners, oj / CPU_BW - 1);
    t.height = imin(CPU_BH, c->n - oi);
    t.width = imin(CPU_BW, c->m - oj);
    t.lm = c->lm; t.slot = bdj;
    lin_tile(&t);
}

/* Full linear-memory fill; returns the exported score (scoring.impala:29-137). */
static int64_t score_linmem(const Scheme* sc, const uint8_t* Q, Index n, const uint8_t* S, Index m,
                            Index* pos_i, Index* pos_j) {
    Vec column = vec_create(n), row = vec_create(m);
    Index nbj_all = round_up_div(m, CPU_BW);
    Vec corners = vec_create(nbj_all - 1);
    V(column, -1) = init_scores(sc, m - 1);
    for (Index i = 0; i < n; ++i) V(column, i) = init_scores(sc, i);
    V(row, -1) = init_scores(sc, n - 1);
    for (Index j = 0; j < m; ++j) V(row, j) = init_scores(sc, j);
    for (Index i = 0; i < nbj_all; ++i) V(corners, i - 1) = init_scores(sc, i * CPU_BW - 1);

    LocalMax lm; LocalMax* lmp = NULL;
    if (sc->kind == SCHEME_LOCAL) {
        Index L = round_up_div(m, CPU_BW);
        lm.max_scores = vec_create(L); lm.max_i = vec_create(L); lm.max_j = vec_create(L);
        for (Index i = 0; i < L; ++i) V(lm.max_scores, i) = SCORE_MIN_VALUE;
        lmp = &lm;
    }

    IterCtx c;
    c.sc = sc; c.Q = Q; c.S = S; c.n = n; c.m = m;
    c.column = &column; c.row = &row; c.corners = &corners; c.lm = lmp;
    c.nbi = round_up_div(n, CPU_BH); c.nbj = nbj_all;
    Index max_blocks = imin(c.nbi, c.nbj);
    Index diags = c.nbi + c.nbj - 1;
    for (Index d = 0; d < diags; ++d) {
        c.d = d;
        Index nb = imin3(d + 1, max_blocks, diags - d);
        parallel_for(0, nb, iter_body, &c);
    }

    int64_t result;
    Index pi = -1, pj = -1;
    if (sc->kind == SCHEME_GLOBAL) {
        result = V(column, n - 1); pi = n - 1; pj = m - 1;
    } else if (sc->kind == SCHEME_SEMIGLOBAL) {
        Score score = SCORE_MIN_VALUE, s2; Index idx;
        reduce_max(&row, -1, row.length + 1, &s2, &idx);
        if (s2 > score) { score = s2; pi = n - 1; pj = idx; }
        reduce_max(&column, -1, column.length + 1, &s2, &idx);
        if (s2 > score) { score = s2; pi = idx; pj = m - 1; }
        result = score;
    } else {
        Score s2; Index idx;
        reduce_max(&lm.max_scores, 0, lm.max_scores.length, &s2, &idx);
        result = s2;
        if (idx >= 0) { pi = V(lm.max_i, idx); pj = V(lm.max_j, idx); }
        free(lm.max_scores.buf); free(lm.max_i.buf); free(lm.max_j.buf);
    }
    if (pos_i) *pos_i = pi;
    if (pos_j) *pos_j = pj;
    free(column.buf); free(row.buf); free(corners.buf);
    return result;
}

/* ----------------------------------------------------- Hirschberg ------- */
/* Splits (traceback_lintime.impala:1-42). */
typedef struct { Vec spl; Index num_blocks; Index bpp; } Splits;

static Score spl_read(Splits* s, Index idx) {
    Score v = V(s->spl, idx);
    if (v == SPLIT_UNSET) {
        g_error = 1;
        fprintf(stderr, "oracle: read of unset split index %d\n", idx);
    }
    return v;
}
static void part_dims(Splits* s, Index part, Index* off, Index* height) {
    Index start = part * s->bpp - 1;
    Index end = imin((part + 1) * s->bpp - 1, s->num_blocks - 1);
    Score o = spl_read(s, start);
    *off = o;
    *height = spl_read(s, end) - o;
}
static void set_split(Splits* s, Index part, Index position) {
    V(s->spl, part * s->bpp + s->bpp / 2 - 1) = position;
}

/* get_sequence_acc_half (traceback_lintime.impala:137-148). */
static SeqAcc seq_half(const uint8_t* base, Index half_offset, Index half_size, Index half_block,
                       Index block_size, int is_left) {
    SeqAcc a; a.base = base;
    if (is_left) { a.off = half_offset + half_block * block_size; a.rev = 0; }
    else { a.off = half_offset + half_size - half_block * block_size - 1; a.rev = 1; }
    return a;
}

typedef struct {
    const Scheme* sc; const uint8_t* Q; const uint8_t* S; Index n, m;
    Splits* splits;
    Vec *col_left, *col_right, *row, *corners;
    Index half, num_halfs, bw, hnbi, hnb, d;
} PartCtx;

static void part_body(void* p, Index bdj) {                 /* iteration_cpu.impala:77-115 */
    PartCtx* c = (PartCtx*)p;
    Index hidx = bdj / c->hnb;
    int left = (hidx % 2) == 0;
    Index hbdj = bdj % c->hnb;
    Index hbi = imin(c->d, c->hnbi - 1) - hbdj;
    Index hbj = imax(c->d - c->hnbi + 1, 0) + hbdj;
    Index hoj = hidx * c->half;
    Index hoi, hh;
    part_dims(c->splits, hidx / 2, &hoi, &hh);
    Index oi = hoi + hbi * CPU_BH;
    Index oj = hoj + hbj * c->bw;
    Index hw = imin(c->half, c->m - hoj);
    Index h = imin(CPU_BH, hh - hbi * CPU_BH);
    Index w = imin(c->bw, c->m - oj);
    if (w > 0) {
        LinTile t;
        t.sc = c->sc;
        t.qa = seq_half(c->Q, hoi, hh, hbi, CPU_BH, left);
        t.sa = seq_half(c->S, hoj, hw, hbj, c->bw, left);
        t.col = left ? c->col_left : c->col_right; t.offset_i = oi;
        t.row = c->row; t.offset_j = oj;
        t.corner = &V(*c->corners, oj / c->bw - 1);
        t.height = h; t.width = w;
        t.lm = NULL; t.slot = 0;
        lin_tile(&t);
    }
}

/* hb_sum (traceback_lintime.impala:44-135). */
static Index hb_sum(const Scheme* sc, Vec* L, Vec* R, Splits* splits, Index n, Index m,
                    Index half, Index parts) {
    Index bwh = imin(CPU_BW, half * 2);
    Index bpp = half * 2 / bwh;
    Index nblk = parts * bpp;
    Score* bmax = (Score*)malloc(sizeof(Score) * (size_t)(nblk > 0 ? nblk : 1));
    Index* bind = (Index*)malloc(sizeof(Index) * (size_t)(nblk > 0 ? nblk : 1));
    for (Index block = 0; block < nblk; ++block) {
        Index part = block / bpp, pb = block % bpp;
        Index po, len;
        part_dims(splits, part, &po, &len);
        Score mx = SCORE_MIN_VALUE; Index index = -1;
        if (pb == 0 && len > 0) {
            Index lhw = half;
            Index rhw = imin(half, m - (part * 2 + 1) * half);
            mx = init_scores(sc, lhw - 1) + V(*R, po + len - 1);
            index = -1;
            Score last = V(*L, po + len - 1) + init_scores(sc, rhw - 1);
            if (last > mx) { mx = last; index = len - 1; }
        }
        for (Index i = pb; i < len - 1; i += bpp) {
            Score val = V(*L, po + i) + V(*R, po + len - i - 2);
            if (val > mx) { mx = val; index = i; }
        }
        bmax[block] = mx; bind[block] = index;
    }
    Vec heights = vec_create(parts * 2 + 1);
    for (Index part = 0; part < parts; ++part) {
        Index bo = part * bpp;
        Index oi, h;
        part_dims(splits, part, &oi, &h);
        Score mx = bmax[bo]; Index index = bind[bo];
        for (Index i = 1; i < bpp; ++i)
            if (bmax[bo + i] > mx) { mx = bmax[bo + i]; index = bind[bo + i]; }
        set_split(splits, part, oi + index + 1);
        V(heights, part * 2) = index + 1;
        V(heights, part * 2 + 1) = h - index - 1;
        if (part == parts - 1) V(heights, parts * 2) = n - (oi + h);
    }
    Score max_h; Index dummy;
    reduce_max(&heights, 0, heights.length, &max_h, &dummy);
    free(bmax); free(bind); free(heights.buf);
    return max_h;
}

/* traceback_lintime_step (align.impala:273-290). */
static Index hb_step(const Scheme* sc, const uint8_t* Q, Index n, const uint8_t* S, Index m,
                     Index pw, Splits* splits, Index max_h) {
    Index half = pw / 2;
    Index num_halfs = (m + half - 1) / pw * 2;
    Index bw = imin(CPU_BW, half);
    /* create_scoring_hb_matrix_linmem (scoring.impala:261-317) */
    Index nbj = round_up_div(m, bw);
    Vec colL = vec_create(n), colR = vec_create(n), row = vec_create(m), corners = vec_create(nbj - 1);
    Index bpp_s = pw / bw;
    for (Index b = 0; b < nbj; ++b) {
        Index part = b / bpp_s, block = b % bpp_s;
        Index oi, ph;
        part_dims(splits, part, &oi, &ph);
        Index part_blocks = imin(bpp_s, nbj - part * bpp_s);
        for (Index i = block; i < ph; i += part_blocks) {
            V(colL, oi + i) = init_scores(sc, i);
            V(colR, oi + i) = init_scores(sc, i);
        }
    }
    for (Index i = 0; i < m; ++i) V(row, i) = init_scores(sc, i % half);
    for (Index i = 0; i < nbj; ++i) V(corners, i - 1) = init_scores(sc, (i * bw) % half - 1);

    /* iteration_partitioned (iteration_cpu.impala:59-119) */
    PartCtx c;
    c.sc = sc; c.Q = Q; c.S = S; c.n = n; c.m = m; c.splits = splits;
    c.col_left = &colL; c.col_right = &colR; c.row = &row; c.corners = &corners;
    c.half = half; c.num_halfs = num_halfs; c.bw = bw;
    Index hnbj = half / bw;
    c.hnbi = round_up_div(max_h, CPU_BH);
    Index hmax = imin(c.hnbi, hnbj);
    Index diags = c.hnbi + hnbj - 1;
    for (Index d = 0; d < diags; ++d) {
        c.d = d;
        c.hnb = imin3(d + 1, hmax, diags - d);
        parallel_for(0, c.hnb * num_halfs, part_body, &c);
    }
    Index new_h = hb_sum(sc, &colL, &colR, splits, n, m, half, num_halfs / 2);
    free(colL.buf); free(colR.buf); free(row.buf); free(corners.buf);
    return new_h;
}

/* Blockwise predecessor fill of one 128-col block (iteration_cpu.impala:121-157,
 * scoring_cpu.impala:125-157, mapping_cpu.impala:67-84). */
typedef struct {
    const Scheme* sc; const uint8_t* Q; const uint8_t* S; Index n, m;
    Splits* splits; Pred* predc; Index pw_mem;
} TbCtx;

#define PRED_AT(predc, off_i, i, j) (predc)[((size_t)((i) + (off_i) + 1)) * 129 + (size_t)((j) + 1)]

static void tb_fill_body(void* p, Index bj) {
    TbCtx* c = (TbCtx*)p;
    const Scheme* sc = c->sc;
    Index oj = bj * MIN_PART_WIDTH_HB;
    Index oi, h;
    part_dims(c->splits, bj, &oi, &h);
    Index w = imin(MIN_PART_WIDTH_HB, c->m - oj);
    Index poff = oi + bj;
    for (Index j = -1; j < w; ++j) PRED_AT(c->predc, poff, -1, j) = init_predc_cols(sc, j);
    for (Index i = 0; i < h; ++i) PRED_AT(c->predc, poff, i, -1) = init_predc_rows(sc, i);
    Score row[MIN_PART_WIDTH_HB + 1];
    for (Index j = -1; j < w; ++j) row[j + 1] = init_scores(sc, j);
    Score no_gap = init_scores(sc, -1), gap_q = 0;
    for (Index i = 0; i < h; ++i) {
        gap_q = init_scores(sc, i);
        uint8_t qs = c->Q[oi + i];
        for (Index j = 0; j < w; ++j) {
            Pred pr;
            Score s = relax(sc, qs, c->S[oj + j], no_gap, gap_q, row[j + 1], &pr);
            PRED_AT(c->predc, poff, i, j) = pr;
            no_gap = row[j + 1];
            gap_q = s;
            row[j + 1] = s;
        }
        no_gap = init_scores(sc, i);
    }
}

/* traceback_offset (traceback.impala:47-80). */
static void traceback_offset(const uint8_t* Q, const uint8_t* S, char* alq, char* als,
                             const Pred* predc, Index poff, Index oq, Index os, Index ei, Index ej) {
    Index i = ei, j = ej;
    Pred pred = PRED_AT(predc, poff, i, j);
    while (pred != PRED_NONE) {
        char sq = '_', ss = '_';
        Index out = i + j + 1;
        if (pred == PRED_NO_GAP || pred == PRED_GAP_S) { sq = (char)Q[oq + i]; --i; }
        if (pred == PRED_NO_GAP || pred == PRED_GAP_Q) { ss = (char)S[os + j]; --j; }
        alq[oq + os + out] = sq;
        als[oq + os + out] = ss;
        pred = PRED_AT(predc, poff, i, j);
    }
}

/* traceback_lintime (align.impala:237-311).  Returns the value the reference
 * returns (scoring.get_score() of a never-relaxed scoring object, §0.2). */
static int64_t construct_lintime(const Scheme* sc, const uint8_t* Q, Index n, const uint8_t* S, Index m,
                                 char* alq, char* als, int32_t* splits_out, Index splits_cap) {
    for (Index i = 0; i < n + m; ++i) { alq[i] = ' '; als[i] = ' '; }   /* traceback.impala:20-23 */
    Index pw = next_pow_2(m);
    Index max_h = n;
    Splits sp;
    sp.num_blocks = round_up_div(m, MIN_PART_WIDTH_HB);
    sp.spl = vec_create(sp.num_blocks);
    for (Index i = -1; i < sp.num_blocks; ++i) V(sp.spl, i) = SPLIT_UNSET;
    sp.bpp = pw / MIN_PART_WIDTH_HB;
    V(sp.spl, -1) = 0;
    if (sp.num_blocks > 0) V(sp.spl, sp.num_blocks - 1) = n;
    while (pw > MIN_PART_WIDTH_HB) {
        max_h = hb_step(sc, Q, n, S, m, pw, &sp, max_h);
        pw /= 2;
        sp.bpp /= 2;
    }
    /* traceback_lintime_trace (align.impala:292-311) */
    Index nbj = sp.num_blocks;
    if (nbj > 0) {
        size_t rows = (size_t)(n + nbj);
        Pred* predc = (Pred*)calloc(rows * 129, 1);
        TbCtx c;
        c.sc = sc; c.Q = Q; c.S = S; c.n = n; c.m = m; c.splits = &sp; c.predc = predc;
        parallel_for(0, nbj, tb_fill_body, &c);
        for (Index b = 0; b < nbj; ++b) {                      /* iteration_tb */
            Index oi, h;
            part_dims(&sp, b, &oi, &h);
            Index oj = b * MIN_PART_WIDTH_HB;
            Index w = imin(MIN_PART_WIDTH_HB, m - oj);
            traceback_offset(Q, S, alq, als, predc, oi + b, oi, oj, h - 1, w - 1);
        }
        free(predc);
    }
    if (splits_out) {
        for (Index i = 0; i < sp.num_blocks && i < splits_cap; ++i) splits_out[i] = V(sp.spl, i);
    }
    free(sp.spl.buf);
    if (sc->kind == SCHEME_GLOBAL) return init_scores(sc, n - 1);
    if (sc->kind == SCHEME_SEMIGLOBAL) return 0;
    return SCORE_MIN_VALUE;
}

/* -------------------------------------------------------- public API ---- */
static Scheme make_scheme(int kind, int match, int mismatch, int gap) {
    Scheme s; s.kind = kind; s.match = match; s.mismatch = mismatch; s.gap = gap; return s;
}

/* Score with general linear parameters; pos_i/pos_j optional (not exported by the ABI). */
int64_t oracle_score(int kind, const char* q, int n, const char* s, int m,
                     int match, int mismatch, int gap, int32_t* pos_i, int32_t* pos_j) {
    Scheme sc = make_scheme(kind, match, mismatch, gap);
    g_error = 0;
    return score_linmem(&sc, (const uint8_t*)q, n, (const uint8_t*)s, m, pos_i, pos_j);
}

/* construct_* with the reference's column-split Hirschberg.  Returns the
 * reference's literal return value; the optimal score is
 * available through oracle_score().  splits_out (optional) receives the final
 * split rows (nb = ceil(m/128) entries). */
int64_t oracle_construct(int kind, const char* q, int n, const char* s, int m,
                         int match, int mismatch, int gap, char* alq, char* als,
                         int32_t* splits_out, int splits_cap) {
    Scheme sc = make_scheme(kind, match, mismatch, gap);
    g_error = 0;
    return construct_lintime(&sc, (const uint8_t*)q, n, (const uint8_t*)s, m, alq, als,
                             splits_out, splits_cap);
}

/* The six ABI-shaped entry points with the fixed (2,-1,-1) scheme (export.impala). */
int64_t oracle_global_alignment_score(const char* q, int n, const char* s, int m) {
    return oracle_score(SCHEME_GLOBAL, q, n, s, m, 2, -1, -1, NULL, NULL);
}
int64_t oracle_semiglobal_alignment_score(const char* q, int n, const char* s, int m) {
    return oracle_score(SCHEME_SEMIGLOBAL, q, n, s, m, 2, -1, -1, NULL, NULL);
}
int64_t oracle_local_alignment_score(const char* q, int n, const char* s, int m) {
    return oracle_score(SCHEME_LOCAL, q, n, s, m, 2, -1, -1, NULL, NULL);
}
int64_t oracle_construct_global_alignment(const char* q, int n, const char* s, int m, char* aq, char* as_) {
    return oracle_construct(SCHEME_GLOBAL, q, n, s, m, 2, -1, -1, aq, as_, NULL, 0);
}
int64_t oracle_construct_semiglobal_alignment(const char* q, int n, const char* s, int m, char* aq, char* as_) {
    return oracle_construct(SCHEME_SEMIGLOBAL, q, n, s, m, 2, -1, -1, aq, as_, NULL, 0);
}
int64_t oracle_construct_local_alignment(const char* q, int n, const char* s, int m, char* aq, char* as_) {
    return oracle_construct(SCHEME_LOCAL, q, n, s, m, 2, -1, -1, aq, as_, NULL, 0);
}

/* construct_*_alignment_fulltb (export.impala:37-53, 93-109, 150-166): all three
 * pass global_scheme(linear_scoring_scheme(2,-1,-1)) (export.impala:52,108,165),
 * so each is traceback_full (align.impala:190-216) of the GLOBAL scheme: one fill of
 * the whole matrix writing every predecessor into a full (n+1) x (m+1) matrix with
 * the scheme's border predecessors (full_predecessors, predecessors.impala:11-34),
 * then traceback_offset (traceback.impala:47-80) from get_score_pos() = (n-1, m-1)
 * (scoring.impala:34) over blank-filled outputs (traceback.impala:14-44).  Returns
 * get_score() = H[n-1][m-1] (the scoring object IS relaxed here, unlike
 * traceback_lintime's).  Memory O(n*m): test sizes only. */
int64_t oracle_construct_fulltb(const char* qc, int n, const char* sc_, int m, int match, int mismatch, int gap,
                                char* alq, char* als) {
    const uint8_t* Q = (const uint8_t*)qc;
    const uint8_t* S = (const uint8_t*)sc_;
    Scheme sc = make_scheme(SCHEME_GLOBAL, match, mismatch, gap);
    g_error = 0;
    const size_t W = (size_t)m + 1;
    uint8_t* P = (uint8_t*)malloc(((size_t)n + 1) * W);
    Score* row = (Score*)malloc(W * sizeof(Score));
    if (!P || !row) { free(P); free(row); g_error = 1; return 0; }
#define PF(i, j) P[((size_t)(i) + 1) * W + (size_t)(j) + 1]
    for (Index j = -1; j < m; ++j) { PF(-1, j) = init_predc_cols(&sc, j); row[j + 1] = init_scores(&sc, j); }
    for (Index i = 0; i < n; ++i) {
        PF(i, -1) = init_predc_rows(&sc, i);
        Score diag = row[0];                 /* H[i-1][-1] */
        row[0] = init_scores(&sc, i);        /* H[i][-1] */
        for (Index j = 0; j < m; ++j) {
            Pred pr;
            const Score v = relax(&sc, Q[i], S[j], diag, row[j], row[j + 1], &pr);
            diag = row[j + 1];
            row[j + 1] = v;
            PF(i, j) = pr;
        }
    }
    const int64_t score = (n > 0 && m > 0) ? row[m] : (n > 0 ? init_scores(&sc, n - 1) : init_scores(&sc, m - 1));
    const size_t L = (size_t)n + (size_t)m;
    memset(alq, ' ', L);
    memset(als, ' ', L);
    Index i = n - 1, j = m - 1;
    Pred pr = PF(i, j);
    while (pr != PRED_NONE) {
        char sq = '_', ss = '_';
        const Index pos = i + j + 1;
        if (pr == PRED_NO_GAP || pr == PRED_GAP_S) { sq = (char)Q[i]; --i; }
        if (pr == PRED_NO_GAP || pr == PRED_GAP_Q) { ss = (char)S[j]; --j; }
        alq[pos] = sq;
        als[pos] = ss;
        pr = PF(i, j);
    }
#undef PF
    free(P);
    free(row);
    return (n == 0 && m == 0) ? 0 : score;
}

/* ===================================================================== */
/* Build-defined affine gap (Gotoh).  NO reference semantics exist        */
/* (affine_scoring_scheme, align.impala:153-166, is dead and broken):     */
/* parity unpinned by the reference; pinned by open == 0 => linear.       */
/*   E[i][j] = max(E[i][j-1] + ge, H[i][j-1] + go + ge)   (GAP_Q, left)    */
/*   F[i][j] = max(F[i-1][j] + ge, H[i-1][j] + go + ge)   (GAP_S, up)      */
/*   H[i][j] = max(H[i-1][j-1] + sub, E, F)  (local: max(., 0))            */
/* Borders: global H[-1][j] = go + (j+1) ge, H[i][-1] = go + (i+1) ge,     */
/* H[-1][-1] = 0; semiglobal/local 0; E[i][-1] = F[-1][j] = -inf.          */
/* Score: global H[n-1][m-1]; semiglobal max(last row incl. -1, last col   */
/* incl. -1); local max cell.  Position (local): max H, then smallest i,   */
/* then smallest j.                                                        */
/* ===================================================================== */
#define AFF_NEG_INF (-(1 << 29))

int64_t oracle_affine_score(int kind, const char* qc, int n, const char* sc_, int m,
                            int match, int mismatch, int go, int ge,
                            int32_t* pos_i, int32_t* pos_j) {
    const uint8_t* q = (const uint8_t*)qc; const uint8_t* s = (const uint8_t*)sc_;
    Score* H = (Score*)malloc(sizeof(Score) * (size_t)(m + 1));
    Score* F = (Score*)malloc(sizeof(Score) * (size_t)(m + 1));
    /* H[-1][j-1] at H[j] */
    H[0] = 0;
    for (Index j = 0; j < m; ++j) H[j + 1] = kind == SCHEME_GLOBAL ? go + (j + 1) * ge : 0;
    for (Index j = 0; j <= m; ++j) F[j] = AFF_NEG_INF;
    Score best = SCORE_MIN_VALUE; Index bi = -1, bj = -1;
    Score lastcol_best = SCORE_MIN_VALUE; Index lc_i = -1;
    if (kind == SCHEME_SEMIGLOBAL) { lastcol_best = 0; lc_i = -1; }
    for (Index i = 0; i < n; ++i) {
        Score diag = H[0];
        Score left = kind == SCHEME_GLOBAL ? go + (i + 1) * ge : 0;
        H[0] = left;
        Score E = AFF_NEG_INF;
        for (Index j = 0; j < m; ++j) {
            Score e1 = E + ge, e2 = left + go + ge;
            E = e1 > e2 ? e1 : e2;
            Score up = H[j + 1];
            Score f1 = F[j + 1] + ge, f2 = up + go + ge;
            Score f = f1 > f2 ? f1 : f2;
            F[j + 1] = f;
            Score h = diag + (q[i] == s[j] ? match : mismatch);
            if (E > h) h = E;
            if (f > h) h = f;
            if (kind == SCHEME_LOCAL && 0 > h) h = 0;
            diag = up;
            H[j + 1] = h;
            left = h;
            if (kind == SCHEME_LOCAL && h > best) { best = h; bi = i; bj = j; }
        }
        if (kind == SCHEME_SEMIGLOBAL && m > 0 && H[m] > lastcol_best) { lastcol_best = H[m]; lc_i = i; }
    }
    int64_t result;
    if (kind == SCHEME_GLOBAL) {
        result = H[m]; bi = n - 1; bj = m - 1;
        if (n == 0) result = m > 0 ? go + m * ge : 0;
        if (m == 0) result = n > 0 ? go + n * ge : 0;
    } else if (kind == SCHEME_SEMIGLOBAL) {
        /* last row incl. index -1 (border 0): first max wins; then the column if strictly greater */
        Score rb = 0; Index rj = -1;
        if (n > 0) for (Index j = 0; j < m; ++j) if (H[j + 1] > rb) { rb = H[j + 1]; rj = j; }
        result = rb; bi = n - 1; bj = rj;
        if (lastcol_best > rb) { result = lastcol_best; bi = lc_i; bj = m - 1; }
    } else {
        result = best;
    }
    if (pos_i) *pos_i = bi;
    if (pos_j) *pos_j = bj;
    free(H); free(F);
    return result;
}

/* ===================================================================== */
/* Build-defined affine CONSTRUCT (linear space).  No reference semantics */
/* (see above); this is the semantics of the HIP path, restated.          */
/*                                                                       */
/* One column-split Hirschberg over the WHOLE matrix (the level / part /  */
/* split structure of the linear construct, align.impala:237-311), where  */
/* the alignment's ends may be free.  Every split boundary b (between     */
/* 128-column blocks b and b+1; -1 = left edge, nb-1 = right edge) holds  */
/* a row spl[b] and a type:                                              */
/*   H      the path crosses b; rows < spl[b] lie left of it;             */
/*   E      same, inside a horizontal gap (opened once, left of b);       */
/*   BEFORE the path ends left of b;  AFTER the path starts right of b.   */
/* Top level: global H .. H (spl -1 .. nb-1 = 0 .. n); local / semiglobal */
/* AFTER .. BEFORE.  A part [sb, eb] is empty if T[sb] = BEFORE or        */
/* T[eb] = AFTER; its start is anchored (H: scheme corner, E: continuing  */
/* gap) or FREE (T[sb] = AFTER), its end anchored (H, or E: ends in a     */
/* gap) or FREE (T[eb] = BEFORE).  FREE means local: zero borders + the   */
/* clamp H >= 0, any cell may end; semiglobal: zero top border (and left  */
/* border at the matrix's left edge), ends on the last row / column.     */
/* Per part: left half forward, right half reversed (free end -> free     */
/* reversed start), then the first maximum (strict >) of                 */
/*   BEFORE (free end):   best end cell in the left half,                 */
/*   AFTER  (free start): best start cell in the right half,              */
/*   rows i = -1 .. len-1: HL(i) + HR(len-i-2), then EL(i) + ER(..) - go. */
/* Final blocks: Gotoh predecessors (H: diag > E > F, local clamp only if */
/* 0 > H; E/F open unless extending is strictly better), walked from the  */
/* block's end (anchored: bottom-right in H or E; free: local first max   */
/* of all cells in row-major order, semiglobal first max of the last row, */
/* then of the last column if strictly greater) back to its start         */
/* (anchored: the corner; free: a clamped cell or the border).  Output in */
/* the sparse i+j+1 layout of traceback.impala:47-80.  Optimal score <= 0 */
/* (local / semiglobal): the empty alignment.                            */
/* ===================================================================== */
enum { BM_NORMAL = 0, BM_EFREE = 1, BM_EPAID = 2, BM_FREE_LOCAL = 3, BM_FREE_SEMI = 4, BM_FREE_SEMI_OPEN = 5 };
enum { T_H = 0, T_E = 1, T_BEFORE = 2, T_AFTER = 3 };
#define ANEG AFF_NEG_INF

typedef struct { const uint8_t* b; Index off; int step; } Acc;
static inline uint8_t acc_at(Acc a, Index i) { return a.b[a.off + (Index)a.step * i]; }
typedef struct { int match, mismatch, go, ge; } AffSc;

/* Border values (H space) of a sub-problem by border mode: corner, top row (c >= 0),
 * left column (r >= 0).  FREE_SEMI: the left border is open only at the matrix edge. */
static inline Score bm_corner(int bm) { return (bm == BM_EFREE || bm == BM_EPAID) ? ANEG : 0; }
static inline Score bm_top(int bm, const AffSc* sc, Index c) {
    if (bm == BM_NORMAL || bm == BM_EPAID) return sc->go + (c + 1) * sc->ge;
    if (bm == BM_EFREE) return (c + 1) * sc->ge;
    return 0;
}
static inline Score bm_left(int bm, const AffSc* sc, Index r) {
    if (bm == BM_NORMAL) return sc->go + (r + 1) * sc->ge;
    if (bm == BM_FREE_LOCAL || bm == BM_FREE_SEMI_OPEN) return 0;
    return ANEG;
}

/* Affine DP of q x s (h x w) under border mode bm (local clamp for FREE_LOCAL).
 * Optional outputs: last column H / E, the maximum over all cells, the maximum
 * over the last row. */
static void aff_fill(Acc q, Index h, Acc s, Index w, const AffSc* sc, int bm, Score* colH, Score* colE,
                     Score* best_all, Score* best_last) {
    Score* H = (Score*)malloc(sizeof(Score) * (size_t)(w + 1));
    Score* F = (Score*)malloc(sizeof(Score) * (size_t)(w + 1));
    const int clamp = bm == BM_FREE_LOCAL;
    H[0] = bm_corner(bm);
    for (Index c = 0; c < w; ++c) { H[c + 1] = bm_top(bm, sc, c); F[c + 1] = ANEG; }
    Score ba = ANEG, bl = ANEG;
    for (Index r = 0; r < h; ++r) {
        Score diag = H[0];
        Score left = bm_left(bm, sc, r);
        H[0] = left;
        Score E = ANEG;
        const uint8_t qs = acc_at(q, r);
        for (Index c = 0; c < w; ++c) {
            Score e1 = E + sc->ge, e2 = left + sc->go + sc->ge;
            E = e1 > e2 ? e1 : e2;
            Score up = H[c + 1];
            Score f1 = F[c + 1] + sc->ge, f2 = up + sc->go + sc->ge;
            Score f = f1 > f2 ? f1 : f2;
            F[c + 1] = f;
            Score hv = diag + (qs == acc_at(s, c) ? sc->match : sc->mismatch);
            if (E > hv) hv = E;
            if (f > hv) hv = f;
            if (clamp && 0 > hv) hv = 0;
            diag = up;
            H[c + 1] = hv;
            left = hv;
            if (hv > ba) ba = hv;
            if (r == h - 1 && hv > bl) bl = hv;
        }
        if (colH) colH[r] = H[w];
        if (colE) colE[r] = w > 0 ? E : ANEG;
    }
    if (best_all) *best_all = ba;
    if (best_last) *best_last = bl;
    free(H); free(F);
}

typedef struct { Score* v; Index n; } IVec;   /* logical index -1 at v[0] */
#define IV(x, i) ((x).v[(i) + 1])

/* Final 128-column block: Gotoh with predecessor bytes (bits 0-1: H source 0 diag,
 * 1 E, 2 F, 3 clamped; bit 2 E extends, bit 3 F extends), walk, sparse output.
 * bm: start border mode; e_end: 0 end in H, 1 end in E (both at the bottom-right
 * corner), 2 free end; semi_lastcol: free semiglobal end, the block holds the
 * matrix's last column. */
enum { AP_DIAG = 0, AP_E = 1, AP_F = 2, AP_NONE = 3 };
/* rows / columns the last construct emitted (tests check them against the kind's rules) */
static int32_t g_last_rect[4] = {0, -1, 0, -1};   /* is, ie, js, je */
static inline void emit_q(Index i) {
    if (g_last_rect[1] < g_last_rect[0]) { g_last_rect[0] = g_last_rect[1] = i; return; }
    if (i < g_last_rect[0]) g_last_rect[0] = i;
    if (i > g_last_rect[1]) g_last_rect[1] = i;
}
static inline void emit_s(Index j) {
    if (g_last_rect[3] < g_last_rect[2]) { g_last_rect[2] = g_last_rect[3] = j; return; }
    if (j < g_last_rect[2]) g_last_rect[2] = j;
    if (j > g_last_rect[3]) g_last_rect[3] = j;
}
static void aff_block_walk(const uint8_t* Q, const uint8_t* S, Index oi, Index h, Index oj, Index w,
                           const AffSc* sc, int bm, int e_end, int kind, int semi_lastcol, char* alq, char* als) {
    if (e_end == 2 && h <= 0) return;   /* free end, no rows: the path ended at the block's corner */
    uint8_t* P = (uint8_t*)calloc((size_t)(h > 0 ? h : 1) * (size_t)(w > 0 ? w : 1), 1);
    Score* H = (Score*)malloc(sizeof(Score) * (size_t)(w + 1));
    Score* F = (Score*)malloc(sizeof(Score) * (size_t)(w + 1));
    const int clamp = bm == BM_FREE_LOCAL;
    const int free_start = bm >= BM_FREE_LOCAL;
    H[0] = bm_corner(bm);
    for (Index c = 0; c < w; ++c) { H[c + 1] = bm_top(bm, sc, c); F[c + 1] = ANEG; }
    Score xb = ANEG; Index xi = h - 1, xj = w - 1;   /* free end: the exit cell */
    Score cb = ANEG; Index ci = -1;                  /* semiglobal: first max of the last column */
    for (Index r = 0; r < h; ++r) {
        Score diag = H[0];
        Score left = bm_left(bm, sc, r);
        H[0] = left;
        Score E = ANEG;
        for (Index c = 0; c < w; ++c) {
            uint8_t pb = 0;
            Score e1 = E + sc->ge, e2 = left + sc->go + sc->ge;
            if (e1 > e2) { E = e1; pb |= 4; } else E = e2;
            Score up = H[c + 1];
            Score f1 = F[c + 1] + sc->ge, f2 = up + sc->go + sc->ge;
            Score f;
            if (f1 > f2) { f = f1; pb |= 8; } else f = f2;
            F[c + 1] = f;
            Score hv = diag + (Q[oi + r] == S[oj + c] ? sc->match : sc->mismatch);
            int hs = AP_DIAG;
            if (E > hv) { hv = E; hs = AP_E; }
            if (f > hv) { hv = f; hs = AP_F; }
            if (clamp && 0 > hv) { hv = 0; hs = AP_NONE; }
            pb |= (uint8_t)hs;
            P[(size_t)r * w + c] = pb;
            diag = up;
            H[c + 1] = hv;
            left = hv;
            if (e_end == 2) {
                if (kind == SCHEME_LOCAL) {
                    if (hv > xb) { xb = hv; xi = r; xj = c; }
                } else {
                    if (r == h - 1 && hv > xb) { xb = hv; xi = r; xj = c; }
                    if (semi_lastcol && c == w - 1 && hv > cb) { cb = hv; ci = r; }
                }
            }
        }
    }
    if (e_end == 2 && kind != SCHEME_LOCAL && semi_lastcol && cb > xb) { xb = cb; xi = ci; xj = w - 1; }
    /* walk: state 0 = H, 1 = E, 2 = F */
    Index i = xi, j = xj;
    int st = e_end == 1 ? 1 : 0;
    const Index base = oi + oj;
    while (i >= 0 || j >= 0) {
        if (i < 0 || j < 0) {
            if (free_start) break;   /* the path starts on the border */
            if (i < 0) { alq[base + i + j + 1] = '_'; als[base + i + j + 1] = (char)S[oj + j]; emit_s(oj + j); --j; continue; }
            alq[base + i + j + 1] = (char)Q[oi + i]; als[base + i + j + 1] = '_'; emit_q(oi + i); --i; continue;
        }
        const uint8_t pb = P[(size_t)i * w + j];
        if (st == 0) {
            const int hs = pb & 3;
            if (hs == AP_NONE) break;   /* local: the path starts after this cell */
            if (hs == AP_DIAG) {
                alq[base + i + j + 1] = (char)Q[oi + i]; als[base + i + j + 1] = (char)S[oj + j];
                emit_q(oi + i); emit_s(oj + j);
                --i; --j;
            } else st = hs == AP_E ? 1 : 2;
        } else if (st == 1) {
            alq[base + i + j + 1] = '_'; als[base + i + j + 1] = (char)S[oj + j]; emit_s(oj + j);
            st = (pb & 4) ? 1 : 0;
            --j;
        } else {
            alq[base + i + j + 1] = (char)Q[oi + i]; als[base + i + j + 1] = '_'; emit_q(oi + i);
            st = (pb & 8) ? 2 : 0;
            --i;
        }
    }
    free(P); free(H); free(F);
}

/* Border mode of a FREE end for the kind: local clamps everywhere; semiglobal opens
 * the side border only at the matrix edge. */
static inline int free_bm(int kind, int at_edge) {
    return kind == SCHEME_LOCAL ? BM_FREE_LOCAL : (at_edge ? BM_FREE_SEMI_OPEN : BM_FREE_SEMI);
}


/* One half fill of a Hirschberg level (the tasks of a level are independent and
 * run on g_threads threads, as the HIP path runs them in one launch). */
typedef struct {
    Acc q, s; Index h, w; int bm; Score *colH, *colE; Score best_all, best_last;
} HalfTask;
typedef struct { HalfTask* t; const AffSc* sc; } HalfCtx;
static void half_body(void* p, Index i) {
    HalfCtx* c = (HalfCtx*)p;
    HalfTask* t = &c->t[i];
    aff_fill(t->q, t->h, t->s, t->w, c->sc, t->bm, t->colH, t->colE, &t->best_all, &t->best_last);
}

/* Part geometry of a Hirschberg level of the build-defined affine construct (round 4,
 * DESIGN.md §3.4): level k has 2^(k-1) parts, part p the 128-column blocks
 * [floor(p nb / P), floor((p+1) nb / P)) with P = 2^(k-1), split at block
 * floor((2p+1) nb / 2P) -- every part at its middle block, so every level fills ~nm / 2^(k-1)
 * cells whatever m is.  When nb is a power of two these are exactly the reference
 * construct's parts (next_pow_2(m) wide, split at half width, align.impala:237-290),
 * which the linear compat construct keeps.  The levels end once no part has 2 blocks. */
typedef struct { Index sb, mid, eb, hoj_l, hoj_r, lw, hw; } AffPart;
static AffPart aff_part(Index nb, Index m, Index P, Index p) {
    AffPart a;
    const Index b0 = p * nb / P, b1 = (p + 1) * nb / P, bm = (2 * p + 1) * nb / (2 * P);
    a.sb = b0 - 1; a.eb = b1 - 1; a.mid = bm - 1;
    a.hoj_l = b0 * MIN_PART_WIDTH_HB; a.hoj_r = bm * MIN_PART_WIDTH_HB;
    a.lw = a.hoj_r - a.hoj_l;
    a.hw = imin(b1 * MIN_PART_WIDTH_HB, m) - a.hoj_r;
    return a;
}

/* Returns the level-1 join value (the optimal score; semiglobal: with the empty
 * alignment's 0) or INT64_MIN when m <= 128 (no level); writes the alignment
 * unless a local / semiglobal level-1 value is <= 0 (the empty alignment). */
static int64_t aff_construct_hb(int kind, const uint8_t* Q, Index n, const uint8_t* S, Index m, const AffSc* sc,
                                char* alq, char* als) {
    const Index nb = round_up_div(m, MIN_PART_WIDTH_HB);
    IVec spl, typ;
    spl.n = nb; typ.n = nb;
    spl.v = (Score*)malloc(sizeof(Score) * (size_t)(nb + 1));
    typ.v = (Score*)malloc(sizeof(Score) * (size_t)(nb + 1));
    for (Index i = -1; i < nb; ++i) { IV(spl, i) = SPLIT_UNSET; IV(typ, i) = T_H; }
    IV(spl, -1) = 0;
    IV(spl, nb - 1) = n;
    if (kind != SCHEME_GLOBAL) { IV(typ, -1) = T_AFTER; IV(typ, nb - 1) = T_BEFORE; }
    Score *LH = (Score*)malloc(sizeof(Score) * (size_t)(n + 1)), *LE = (Score*)malloc(sizeof(Score) * (size_t)(n + 1));
    Score *RH = (Score*)malloc(sizeof(Score) * (size_t)(n + 1)), *RE = (Score*)malloc(sizeof(Score) * (size_t)(n + 1));
    HalfTask* tasks = (HalfTask*)malloc(sizeof(HalfTask) * (size_t)(2 * nb + 2));
    Index* tpart = (Index*)malloc(sizeof(Index) * (size_t)(nb + 1));   /* part -> its first task, -1: none */
    int64_t score = INT64_MIN;
    int level1 = 1;
    for (Index P = 1; P < nb; P *= 2) {   /* level k: P = 2^(k-1) parts (nb > 1) */
        const Index parts = P;
        Index nt = 0;
        for (Index p = 0; p < parts; ++p) {   /* this level's half fills */
            const AffPart a = aff_part(nb, m, P, p);
            const int ts = IV(typ, a.sb), te = IV(typ, a.eb);
            tpart[p] = -1;
            if (a.lw <= 0 || a.hw <= 0) continue;   /* a one-block part: no split */
            if (ts == T_BEFORE || te == T_AFTER) continue;
            if (IV(spl, a.sb) == SPLIT_UNSET || IV(spl, a.eb) == SPLIT_UNSET) { g_error = 1; continue; }
            const Index off = IV(spl, a.sb), len = IV(spl, a.eb) - off;
            if (len <= 0) continue;
            tpart[p] = nt;
            HalfTask* L = &tasks[nt++];
            L->q = (Acc){Q, off, 1}; L->s = (Acc){S, a.hoj_l, 1}; L->h = len; L->w = a.lw;
            L->bm = ts == T_H ? BM_NORMAL : ts == T_E ? BM_EFREE : free_bm(kind, a.hoj_l == 0);
            L->colH = LH + off; L->colE = LE + off;
            HalfTask* R = &tasks[nt++];
            R->q = (Acc){Q, off + len - 1, -1}; R->s = (Acc){S, a.hoj_r + a.hw - 1, -1}; R->h = len; R->w = a.hw;
            R->bm = te == T_H ? BM_NORMAL : te == T_E ? BM_EPAID : free_bm(kind, a.hoj_r + a.hw == m);
            R->colH = RH + off; R->colE = RE + off;
        }
        HalfCtx hc = {tasks, sc};
        parallel_for(0, nt, half_body, &hc);
        for (Index p = 0; p < parts; ++p) {   /* joins */
            const AffPart a = aff_part(nb, m, P, p);
            if (a.lw <= 0 || a.hw <= 0) continue;
            const Index sb = a.sb, eb = a.eb, mid = a.mid;
            const int ts = IV(typ, sb), te = IV(typ, eb);
            if (ts == T_BEFORE || te == T_AFTER) {   /* empty part: so are both halves */
                IV(typ, mid) = ts == T_BEFORE ? T_BEFORE : T_AFTER;
                IV(spl, mid) = IV(spl, sb);
                continue;
            }
            if (IV(spl, sb) == SPLIT_UNSET || IV(spl, eb) == SPLIT_UNSET) { g_error = 1; continue; }
            const Index off = IV(spl, sb), len = IV(spl, eb) - off;
            const Index hoj_l = a.hoj_l, hoj_r = a.hoj_r, hw = a.hw;
            const int lbm = ts == T_H ? BM_NORMAL : ts == T_E ? BM_EFREE : free_bm(kind, hoj_l == 0);
            const int rbm = te == T_H ? BM_NORMAL : te == T_E ? BM_EPAID : free_bm(kind, hoj_r + hw == m);
            const int sfree = ts == T_AFTER, efree = te == T_BEFORE;
            Score bestL = ANEG, bestR = ANEG;
            if (tpart[p] >= 0) {
                const HalfTask* L = &tasks[tpart[p]];
                const HalfTask* R = L + 1;
                if (efree) bestL = kind == SCHEME_LOCAL ? L->best_all : L->best_last;
                if (sfree) bestR = kind == SCHEME_LOCAL ? R->best_all : R->best_last;
            }
            /* index -1: the halves' top borders at the midline (a FREE top border is no gap) */
            const Score bLH = bm_top(lbm, sc, a.lw - 1), bLE = sfree ? ANEG : bLH;
            const Score bRH = bm_top(rbm, sc, hw - 1), bRE = efree ? ANEG : bRH;
            Score best = SCORE_MIN_VALUE; Index idx = -1; int type = T_H;
            if (efree && bestL > best) { best = bestL; type = T_BEFORE; }
            if (sfree && bestR > best) { best = bestR; type = T_AFTER; }
            for (Index i = -1; i < len; ++i) {
                const Index k = len - i - 2;
                const Score hl = i < 0 ? bLH : LH[off + i], el = i < 0 ? bLE : LE[off + i];
                const Score hr = k < 0 ? bRH : RH[off + k], er = k < 0 ? bRE : RE[off + k];
                Score v = hl + hr;
                if (v > best) { best = v; idx = i; type = T_H; }
                v = el + er - sc->go;
                if (v > best) { best = v; idx = i; type = T_E; }
            }
            IV(typ, mid) = type;
            IV(spl, mid) = type == T_BEFORE ? off + len : type == T_AFTER ? off : off + idx + 1;
            if (level1 && p == 0) score = kind == SCHEME_SEMIGLOBAL && best < 0 ? 0 : best;
        }
        if (level1 && kind != SCHEME_GLOBAL && score <= 0) goto done;   /* the empty alignment */
        level1 = 0;
    }
    for (Index b = 0; b < nb; ++b) {
        const int ts = IV(typ, b - 1), te = IV(typ, b);
        if (ts == T_BEFORE || te == T_AFTER) continue;
        const Index oi = IV(spl, b - 1), h = IV(spl, b) - oi;
        const Index oj = b * MIN_PART_WIDTH_HB, w = imin(MIN_PART_WIDTH_HB, m - oj);
        if (IV(spl, b - 1) == SPLIT_UNSET || IV(spl, b) == SPLIT_UNSET) { g_error = 1; continue; }
        const int bm = ts == T_H ? BM_NORMAL : ts == T_E ? BM_EFREE : free_bm(kind, oj == 0);
        const int e_end = te == T_H ? 0 : te == T_E ? 1 : 2;
        aff_block_walk(Q, S, oi, h, oj, w, sc, bm, e_end, kind, oj + w == m, alq, als);
    }
done:
    free(spl.v); free(typ.v); free(LH); free(LE); free(RH); free(RE); free(tasks); free(tpart);
    return score;
}

/* Rectangle [is, ie] x [js, je] of the last oracle_affine_construct (ie < is: empty). */
void oracle_affine_last_rect(int32_t* rect) { memcpy(rect, g_last_rect, sizeof g_last_rect); }

int64_t oracle_affine_construct(int kind, const char* qc, int n, const char* sc_, int m, int match, int mismatch,
                                int go, int ge, char* alq, char* als) {
    for (Index i = 0; i < n + m; ++i) { alq[i] = ' '; als[i] = ' '; }
    g_last_rect[0] = 0; g_last_rect[1] = -1; g_last_rect[2] = 0; g_last_rect[3] = -1;
    AffSc sc = {match, mismatch, go, ge};
    /* the score: the level-1 join of the Hirschberg (m > 128), else one score fill */
    if (n > 0 && m > MIN_PART_WIDTH_HB)
        return aff_construct_hb(kind, (const uint8_t*)qc, n, (const uint8_t*)sc_, m, &sc, alq, als);
    const int64_t score = oracle_affine_score(kind, qc, n, sc_, m, match, mismatch, go, ge, NULL, NULL);
    if (n + m == 0) return score;
    if (kind != SCHEME_GLOBAL && (score <= 0 || n == 0 || m == 0)) return score;   /* the empty alignment */
    if (m == 0) {   /* global: all query rows against gaps, down the left border: position i + (-1) + 1 */
        for (Index i = 0; i < n; ++i) { alq[i] = qc[i]; als[i] = '_'; emit_q(i); }
    } else {
        aff_construct_hb(kind, (const uint8_t*)qc, n, (const uint8_t*)sc_, m, &sc, alq, als);
    }
    return score;
}
