"""Shared graph builders for the parity tests (seeded, deterministic)."""
import numpy as np


def chain_text(n):
    return "".join(f"{i} {i + 1}\n" for i in range(n - 1)).encode()


def random_graph(rng, kind, n):
    """Directed multigraph edges (src, dst) of a few shapes the reference's fuzz used
    (uniform, power-law hub, chain + noise)."""
    if kind == "uniform":
        m = int(rng.integers(0, 6 * n + 1))
        return rng.integers(0, n, m), rng.integers(0, n, m)
    if kind == "hub":
        m = 8 * n
        a = rng.zipf(1.6, m) % n
        b = rng.integers(0, n, m)
        flip = rng.random(m) < 0.5
        return np.where(flip, a, b), np.where(flip, b, a)
    if kind == "chain":
        s = np.arange(n - 1)
        noise = max(1, n // 20)
        return (np.concatenate([s, rng.integers(0, n, noise)]),
                np.concatenate([s + 1, rng.integers(0, n, noise)]))
    raise ValueError(kind)


def to_text(src, dst, w=None, style=0):
    """Edge-list text in a few of the layouts the reference accepts."""
    lines = ["# FromNodeId\tToNodeId\n"] if style else []
    for i, (a, b) in enumerate(zip(src, dst)):
        sep = "\t" if (style == 0 or i % 3) else "  "
        tail = f"\t{w[i]}" if w is not None else ""
        eol = "\r\n" if (style == 2 and i % 2) else "\n"
        lines.append(f"{a}{sep}{b}{tail}{eol}")
        if style and i % 97 == 0:
            lines.append("\n# comment line\n")
    return "".join(lines).encode()


def csr_to_text(row, col):
    """SNAP-style edge list (tab-separated, '#' header) of a CSR, rows in order."""
    import numpy as np
    src = np.repeat(np.arange(len(row) - 1, dtype=np.int64), np.diff(row))
    body = np.char.add(np.char.add(src.astype(str), "\t"), np.asarray(col, dtype=np.int64).astype(str))
    return ("# Directed graph (synthetic, web-Google-shaped)\n# FromNodeId\tToNodeId\n" +
            "\n".join(body.tolist()) + "\n").encode()
