"""Loss-curve plotting (reference plot.ipynb:25-49, 68).

Parses ``"{step} {train|val} {loss}"`` lines (the log/log.txt format written by the trainer and by the
reference's train.py) and saves train-vs-val curves to a PNG; ``--hellaswag`` draws the reference's
0.324 line for comparison when a HellaSwag result file is given.

  python -m mamba_distributed_amd.utils.plot log/log.txt -o log/validation_loss.png
"""
from __future__ import annotations

import argparse
from typing import Dict, List, Tuple


def parse_log(path: str) -> Dict[str, Tuple[List[int], List[float]]]:
    out: Dict[str, Tuple[List[int], List[float]]] = {"train": ([], []), "val": ([], [])}
    with open(path) as f:
        for line in f:
            parts = line.split()
            if len(parts) != 3 or parts[1] not in out:
                continue
            out[parts[1]][0].append(int(parts[0]))
            out[parts[1]][1].append(float(parts[2]))
    return out


def plot(path: str, out_png: str, title: str = "Mamba training", ref_log: str = None):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    d = parse_log(path)
    fig, ax = plt.subplots(figsize=(10, 5))
    ax.plot(*d["train"], label="train loss", alpha=0.7)
    ax.plot(*d["val"], "o-", label="val loss")
    if ref_log:
        r = parse_log(ref_log)
        ax.plot(*r["val"], "s--", label="reference val loss", alpha=0.7)
    ax.set_xlabel("step")
    ax.set_ylabel("loss")
    ax.set_title(title)
    ax.legend()
    ax.grid(alpha=0.3)
    fig.tight_layout()
    fig.savefig(out_png, dpi=120)
    return out_png


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("log")
    p.add_argument("-o", "--out", default="log/validation_loss.png")
    p.add_argument("--ref-log", default=None, help="overlay another log (e.g. the reference's log_mamba.txt)")
    a = p.parse_args(argv)
    print(plot(a.log, a.out, ref_log=a.ref_log))


if __name__ == "__main__":
    main()
