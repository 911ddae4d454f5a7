"""Write a word2vec test corpus: one sentence of integer word ids per line.

Same shape of corpus as the reference's src/tools/gen-word2vec-data.py
(10,000 lines of 6-15 ids drawn from 0..300), parameterised:

    python tools/gen_word2vec_data.py out.txt [--lines 10000] [--vocab 301]
        [--min-len 6] [--max-len 15] [--seed 0] [--zipf 0]

``--zipf s`` (s > 1) draws ids from a Zipf law instead of uniformly."""
import argparse

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--lines", type=int, default=10000)
    ap.add_argument("--vocab", type=int, default=301)
    ap.add_argument("--min-len", type=int, default=6)
    ap.add_argument("--max-len", type=int, default=15)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--zipf", type=float, default=0.0)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    with open(a.out, "w") as f:
        for _ in range(a.lines):
            n = int(rng.integers(a.min_len, a.max_len + 1))
            if a.zipf > 1:
                ids = (rng.zipf(a.zipf, n) - 1) % a.vocab
            else:
                ids = rng.integers(0, a.vocab, n)
            f.write(" ".join(str(int(i)) for i in ids) + "\n")


if __name__ == "__main__":
    main()
