# Per iteration of an N4_DUMP_D file (oracle/n4_oracle.c dev hook): how often the float mu of S7 moves
# (a step leaves mu unchanged when |p - mu| / N is below half an ulp), and per 1024-block split how many
# blocks never move -- the frozen iterations where PC hits its round caps.
import numpy as np, struct
import sys
f = open(sys.argv[1], 'rb')
its = []
while True:
    h = f.read(8)
    if not h: break
    n = struct.unpack('q', h)[0]
    d = np.frombuffer(f.read(4 * n), np.float32)
    its.append(d)
for it in (5, 14, 15, 16, 17, 18):
    d = its[it - 1]
    p = np.exp(d.astype(np.float64)).astype(np.float32)
    n = len(d)
    mu = np.float32(0)
    N = np.float32(0)
    changes = np.zeros(n, bool)
    mus = np.empty(n, np.float32)
    for k in range(n):
        N = np.float32(np.float64(N) + 1.0)
        Nd = np.float64(N); r = 1.0 / Nd
        A = 1.0 - r; B = np.float64(np.float32(np.float64(p[k]) * r))
        m1 = np.float32(np.float64(mu) * A + B)
        changes[k] = m1 != mu
        mu = m1
        mus[k] = mu
    blk = n // 1024
    moves = changes[:blk * 1024].reshape(1024, blk).sum(1)
    print(f"it {it}: |d| mean {np.abs(d).mean():.2e} max {np.abs(d).max():.2e}, p-1 std {np.std(p.astype(np.float64)-1):.2e}; "
          f"mu final {mus[-1]:.8f}; changes {changes.sum()} of {n}; last change at {np.nonzero(changes)[0][-1]}; "
          f"blocks with 0 moves {int((moves == 0).sum())}, median moves {np.median(moves)}")
