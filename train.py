"""Training entry point — `torchrun --standalone --nproc_per_node=8 train.py` (reference train.py).

With no flags this reproduces the reference run (Mamba-1 280M, 524,288 tok/step, 19,073 steps,
data from ./edu_fineweb10B).  Flags (all optional) select the model preset / mixer, sizes,
synthetic data, a shorter run, DDP knobs and resume.  See mamba_distributed_amd/trainer.py.

  torchrun --standalone --nproc_per_node=8 train.py --model mamba2-280m --synthetic --steps 50
  python train.py --model mamba2-tiny --synthetic --B 2 --T 128 --total-batch-size 512 --steps 5
"""
import argparse
import dataclasses

from mamba_distributed_amd.trainer import TrainArgs, Trainer


def parse_args(argv=None) -> TrainArgs:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    for f in dataclasses.fields(TrainArgs):
        name = "--" + f.name.replace("_", "-")
        default = f.default
        if f.type in ("bool", bool):
            p.add_argument(name, action=argparse.BooleanOptionalAction, default=default)
        else:
            typ = {"int": int, "float": float, "str": str}.get(str(f.type).replace("Optional[", "").rstrip("]"), str)
            p.add_argument(name, type=typ, default=default)
    ns = p.parse_args(argv)
    return TrainArgs(**{f.name: getattr(ns, f.name) for f in dataclasses.fields(TrainArgs)})


if __name__ == "__main__":
    Trainer(parse_args()).run()
