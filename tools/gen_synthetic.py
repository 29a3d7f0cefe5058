"""Synthetic N x L protein families (the generator used for
the reference's measured baselines in BASELINE.md §2).

A root sequence of L residues drawn from the 20 amino acids with defined
PAM entries is mutated once per output sequence: each root position is
deleted with probability p_indel/2, preceded by a random insertion with
probability p_indel/2, and substituted with probability p_sub.
CPython's random.Random (MT19937) makes the output deterministic per seed.
"""
import argparse
import random

AA = "ACDEFGHIKLMNPQRSTVWY"


def gen(n, length, seed, p_sub, p_indel):
    r = random.Random(seed)
    root = [r.choice(AA) for _ in range(length)]
    out = []
    for _ in range(n):
        s = []
        for c in root:
            x = r.random()
            if x < p_indel / 2:
                continue
            if x < p_indel:
                s.append(r.choice(AA))
            s.append(r.choice(AA) if r.random() < p_sub else c)
        out.append("".join(s))
    return out


def to_fasta(seqs):
    return "".join(">syn%d\n%s\n" % (i, s) for i, s in enumerate(seqs))


# name -> (n, L, seed, p_sub, p_indel); BASELINE.json configs 2 and 5 plus the
# two extra survey points.
PRESETS = {
    "syn4x200_s1": (4, 200, 1, 0.10, 0.02),
    "syn8x400_s5": (8, 400, 5, 0.03, 0.002),
    "syn8x400_s11": (8, 400, 11, 0.01, 0.0),
    "syn8x100_s3": (8, 100, 3, 0.05, 0.01),
}


def preset_fasta(name):
    return to_fasta(gen(*PRESETS[name]))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("preset", nargs="?", choices=sorted(PRESETS))
    ap.add_argument("--n", type=int)
    ap.add_argument("--length", type=int)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--p-sub", type=float, default=0.1)
    ap.add_argument("--p-indel", type=float, default=0.02)
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    text = preset_fasta(a.preset) if a.preset else to_fasta(
        gen(a.n, a.length, a.seed, a.p_sub, a.p_indel))
    if a.out:
        open(a.out, "w").write(text)
    else:
        print(text, end="")
