"""shard_plan — host-side arithmetic of the column-block sharded fill.

Pure Python, no GPU: the partition, the shard frames and the split-row combine
that anyseq_amd/csrc/anyseq_shard.cpp implements in C++ (setup_shard,
enqueue_combine, shard_combine_kernel).  tests/test_shard_plan.py drives this
plan over world_size-2 ``gloo`` process groups with a CPU stand-in for the fill,
checking that the decomposition reproduces the oracle's scores.

Frames.  Shard g owns subject columns [c0_g, c0_g + w_g).  Its fill sees the
scheme's top border (H[-1][c] = (c+1) gap for global), so its values are the true
ones shifted by c0_g * gap (global; semiglobal and local borders are 0 and need
no shift).  A left column received from shard g-1 therefore moves into shard g's
frame by + w_{g-1} * (-gap); the bottom front runs on the reversed sequences and
receives from shard g+1, shifted by + w_{g+1} * (-gap).
"""
from __future__ import annotations

NCOMMS = 4          # RCCL communicators: top/bottom direction x link parity
GLOBAL, SEMIGLOBAL, LOCAL = 0, 1, 2


def block(g: int, nshards: int, m: int):
    """(c0, w) of shard g: balanced contiguous column blocks (anyseq_shard.cpp block_c0)."""
    c0 = g * m // nshards
    return c0, (g + 1) * m // nshards - c0


def fronts(n: int):
    """Rows of the top (forward) and bottom (reversed) fronts: the split is at n // 2."""
    h1 = n // 2
    return h1, n - h1


def left_shift_top(kind: int, g: int, nshards: int, m: int, gap: int) -> int:
    """Added to the values received from shard g-1 (top front)."""
    if kind != GLOBAL or g == 0:
        return 0
    return block(g - 1, nshards, m)[1] * -gap


def left_shift_bottom(kind: int, g: int, nshards: int, m: int, gap: int) -> int:
    """Added to the values received from shard g+1 (bottom front, reversed)."""
    if kind != GLOBAL or g == nshards - 1:
        return 0
    return block(g + 1, nshards, m)[1] * -gap


def combine_adjust(kind: int, g: int, nshards: int, m: int, gap: int) -> int:
    """Top frame + bottom frame -> true score: (c0 + (m - c0 - w)) * gap for global."""
    if kind != GLOBAL:
        return 0
    return (m - block(g, nshards, m)[1]) * gap


def split_columns(g: int, nshards: int, w: int):
    """Local split columns j of shard g's combine: [-1, w-1), plus w-1 on the last shard."""
    return range(-1, w if g == nshards - 1 else w - 1)


def chunk_rows_for(h: int) -> int:
    """Rows per transported chunk of a front of h rows (anyseq_shard.cpp chunk_rows):
    1024, doubled while 256 chunks would not cover h, at most 16384."""
    c = 1024
    while c < 16384 and c * 256 < h:
        c *= 2
    return c


def chunks(h: int, chunk_rows: int = 0):
    """Row chunks [r0, r1) shipped per message, and the band count each waits for
    (chunk_rows 0: the engine's adaptive size)."""
    chunk_rows = chunk_rows or chunk_rows_for(h)
    out = []
    for r0 in range(0, h, chunk_rows):
        r1 = min(h, r0 + chunk_rows)
        out.append((r0, r1, (r1 + 63) // 64))
    return out


# ---------------------------------------------------------------- construct --
# Sharded affine construct (anyseq_engine.cpp aff_construct_hb with a
# ConstructShards): the half fills of a Hirschberg level are numbered in part order
# (part p's left half 2k, right half 2k+1 over the non-empty parts) and dealt
# round-robin; so are the final 128-column blocks.  A rank fills only its halves'
# rows of the level's columns (zero elsewhere), a SUM all-reduce assembles them, a
# MAX all-reduce the free-end best cells, and a byte-wise MAX merges the ranks'
# output strings (blanks ' ' are below every written byte).

def half_owner(half_index: int, world: int) -> int:
    return half_index % world


def block_owner(block: int, world: int) -> int:
    return block % world


def level_halves(parts):
    """(half_index, part, side, off, len) of a level's half fills; `parts` lists
    (off, len) per part, None for an empty part (no fill)."""
    out = []
    k = 0
    for p, pr in enumerate(parts):
        if pr is None or pr[1] <= 0:
            continue
        off, ln = pr
        out.append((k, p, "left", off, ln))
        out.append((k + 1, p, "right", off, ln))
        k += 2
    return out


# Column-blocked level 1 (anyseq_shard.cpp level1_setup).  Level 1's two
# halves, transposed (subject as rows), are the two fronts of one problem split at row
# `half`; rank g fills query columns [c0, c0 + w) of both with the boundary-column
# transport above.  Its bottom rows are its segments of the level's columns.

def level1_segments(g: int, world: int, n: int):
    """((first, w) of LH, (first, w) of RH) written by rank g: LH is indexed by query
    position, RH (the reversed half) by distance from the query's end."""
    c0, w = block(g, world, n)
    return (c0, w), (n - c0 - w, w)


def level1_frame(kind: int, first: int, gap: int) -> int:
    """H_true = H_block + this: a global block's top border is the scheme's from its own
    column 0 (the score's frames, `combine_adjust`); free borders are 0 everywhere."""
    return first * gap if kind == GLOBAL else 0


def level1_best_ranks(world: int):
    """Ranks holding the last column of (forward, reversed) half: a last-column best
    cell (semiglobal free end) is theirs alone; every rank's cells count for local."""
    return world - 1, 0


# Column-blocked levels beyond level 1 (anyseq_engine.cpp): level k has
# P = 2^(k-1) parts and is column-blocked when world >= 2P; part p runs over the ranks
# [p*world/P, (p+1)*world/P) exactly like level 1 over all ranks, on its own query rows
# [off, off+len) and subject columns.

def blocked_level(parts: int, world: int) -> bool:
    """Whether a level of `parts` parts is column-blocked over `world` ranks."""
    return world >= 2 * parts


def level1_blocked(n: int, m: int, world: int) -> bool:
    """Whether the engine column-blocks level 1 of an n x m affine construct over `world`
    ranks (anyseq_engine.cpp aff_construct_hb, with transposed halves and enough hardware
    queues): a level exists (m > 128, two 128-column blocks), world >= 2 (the one part over
    all ranks) and the part's query rows -- all n of them at level 1 -- give every rank
    at least one column (len >= G)."""
    return m > 128 and blocked_level(1, world) and n >= world


def part_subgroup(p: int, parts: int, world: int):
    """(first rank, ranks) of part p's subgroup."""
    r0 = p * world // parts
    return r0, (p + 1) * world // parts - r0


def part_segments(rank: int, r0: int, G: int, off: int, length: int):
    """((first, w) of LH, (first, w) of RH) written by `rank` of a part's subgroup: its
    block of the part's query rows, LH indexed by query position, RH by the reversed
    half's column (distance from the part's end, plus off)."""
    c0, w = block(rank - r0, G, length)
    return (off + c0, w), (off + length - c0 - w, w)
