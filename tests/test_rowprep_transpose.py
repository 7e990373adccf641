"""CPU: the bit-matrix transpose k_n4_rowprep uses to turn 16 column bitmap words (bit k = row
32 w + k of one column) into 32 16-bit row pieces (bit i = column c0 + i of one row) --
vent_analysis_amd/csrc/n4.hip, bit_swap_stage / k_n4_rowprep -- restated step for step and checked
against the direct definition, with the tile-row counts and offsets it feeds (k_n4_rowcount's
popcounts, k_n4_rowscan's tile-major exclusive scan, k_n4_rrank's raster ranks).  The GPU parity
tests check the kernel itself end to end (every N4 test goes through it)."""
import numpy as np

M32 = 0xFFFFFFFF


def swap_stage(A, J, m):
    """bit_swap_stage<J>: rows k and k + J (k with bit J clear) swap their J-bit blocks."""
    for k0 in range(0, 32, 2 * J):
        for k in range(k0, k0 + J):
            tt = ((A[k] >> J) ^ A[k + J]) & m
            A[k] ^= (tt << J) & M32
            A[k + J] ^= tt


def rowprep_transpose(words16):
    """16 column words -> 32 row pieces, as the kernel does: the first stage (J = 16, columns 16..31
    zero) is a split, then four masked-shift stages."""
    A = [0] * 32
    for i in range(16):
        A[i] = words16[i] & 0xFFFF
        A[i + 16] = words16[i] >> 16
    swap_stage(A, 8, 0x00FF00FF)
    swap_stage(A, 4, 0x0F0F0F0F)
    swap_stage(A, 2, 0x33333333)
    swap_stage(A, 1, 0x55555555)
    return A


def test_transpose_matches_definition():
    rng = np.random.default_rng(7)
    for trial in range(200):
        dens = (0.0, 0.02, 0.5, 0.98, 1.0)[trial % 5]
        bits = rng.random((16, 32)) < dens            # [column, row]
        words = [int(sum(1 << k for k in range(32) if bits[c, k])) for c in range(16)]
        A = rowprep_transpose(words)
        for k in range(32):
            want = sum(1 << i for i in range(16) if bits[i, k])
            assert A[k] == want, (trial, k)


def test_counts_offsets_and_raster_ranks():
    """The (tile, row) masks assembled from 16-column quarters give k_n4_rowcount's counts; the
    exclusive scan in tile-major order gives the compact offsets; row totals scanned over rows plus
    the running count over the tiles give the raster rank of each (tile, row)'s first voxel."""
    rng = np.random.default_rng(3)
    R, CZ = 70, 192                                  # 3 tiles of 64 columns, a ragged last word
    mask = rng.random((R, CZ)) < 0.3
    ntiles, nw = CZ // 64, (R + 31) // 32
    colbits = np.zeros((nw, CZ), np.uint64)
    for x in range(R):
        colbits[x >> 5] |= (mask[x].astype(np.uint64) << np.uint64(x & 31))
    rowmask = np.zeros((ntiles, R), np.uint64)
    for w in range(nw):
        for g in range(ntiles * 4):                  # one thread's 16 columns of one word
            A = rowprep_transpose([int(colbits[w, 16 * g + i]) for i in range(16)])
            for k in range(32):
                x = 32 * w + k
                if x < R:
                    rowmask[g >> 2, x] |= np.uint64(A[k]) << np.uint64(16 * (g & 3))
    for t in range(ntiles):
        for x in range(R):
            want = sum(1 << j for j in range(64) if mask[x, 64 * t + j])
            assert int(rowmask[t, x]) == want
    cnt = np.array([[bin(int(rowmask[t, x])).count("1") for x in range(R)] for t in range(ntiles)])
    rs = np.concatenate([[0], np.cumsum(cnt.ravel())[:-1]]).reshape(ntiles, R)
    rowbase = np.concatenate([[0], np.cumsum(cnt.sum(axis=0))[:-1]])
    rr = rowbase[None, :] + np.concatenate([np.zeros((1, R), int), np.cumsum(cnt, axis=0)[:-1]])
    # raster rank = masked voxels before (x, first column of tile t) in row-major (x, column) order
    flat = mask.ravel()
    before = np.concatenate([[0], np.cumsum(flat)[:-1]])
    for t in range(ntiles):
        for x in range(R):
            assert rr[t, x] == before[x * CZ + 64 * t]
    # compact offsets: tile-major, row by row inside a tile
    order = [(t, x) for t in range(ntiles) for x in range(R)]
    run = 0
    for t, x in order:
        assert rs[t, x] == run
        run += cnt[t, x]
