"""Pinned hipBLASLt / rocBLAS solution choice for the plain GEMMs (in_proj, out_proj, lm_head).

The projections are tall-skinny bf16 GEMMs with K = 768 / 1536 — a regime where the library's
default heuristic often picks a 256x256x32 macro-tile that leaves the MFMA pipes half idle.
PyTorch's TunableOp benchmarks every hipBLASLt and rocBLAS solution for each (op, shape) it
meets and records the winner in a CSV keyed by the exact GEMM signature; we ship that table
for gfx950 (``tuned/tunableop_gfx950.csv``, produced on an MI355X by ``scripts/tune_gemms.py``)
and replay it read-only at run time.  Shapes that are not in the table fall through to the
library default, so a stale or missing table never changes results — only speed.

The reference has no equivalent (it relies on cuBLAS heuristics under torch.compile);
this is the MI355X-side replacement for compile-time kernel selection.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_TABLE = os.path.join(os.path.dirname(HERE), "tuned", "tunableop_gfx950.csv")


def _arch() -> str:
    try:
        return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]
    except Exception:  # noqa: BLE001 - no device
        return ""


def enable_tuned_gemms(path: Optional[str] = None, tune: bool = False, max_tuning_ms: int = 30) -> bool:
    """Turn on TunableOp.  ``tune=False`` replays ``path`` (default: the shipped gfx950 table);
    ``tune=True`` searches unseen shapes and writes them to ``path`` at exit / on flush.
    Returns True if a table is active.  Env ``MAMBA_AMD_TUNED_GEMMS=0`` disables it."""
    if os.environ.get("MAMBA_AMD_TUNED_GEMMS", "1") == "0" or not torch.cuda.is_available():
        return False
    path = path or os.environ.get("MAMBA_AMD_GEMM_TABLE") or DEFAULT_TABLE  # env: A/B of another table
    if not tune and (not os.path.exists(path) or _arch() != "gfx950"):
        return False
    # The table is keyed by GEMM signatures recorded at the default fp32 matmul precision.  With
    # torch.set_float32_matmul_precision("high") (the reference's A100/TF32 setting) the replayed
    # solutions compute garbage on ROCm 7 / gfx950 (measured: a 280M forward collapses to loss = ln V and
    # the first backward is NaN; the same run without the table, or at "highest", trains).  gfx950 has no
    # xf32 MFMA, so "high" buys nothing: replay always runs at "highest".
    if torch.get_float32_matmul_precision() != "highest":
        import warnings
        warnings.warn("enable_tuned_gemms: forcing torch.set_float32_matmul_precision('highest') "
                      "(the gfx950 solution table is only valid there; gfx950 has no TF32/xf32 mode)")
        torch.set_float32_matmul_precision("highest")
    tunable = torch.cuda.tunable
    tunable.enable(True)
    tunable.set_filename(path)
    tunable.tuning_enable(tune)
    # replay is read-only: never rewrite the shipped table at exit (every DDP rank would race on it);
    # older torch has no switch and only writes when tuning found new results
    if hasattr(tunable, "write_file_on_exit"):
        tunable.write_file_on_exit(bool(tune))
    if tune:
        tunable.set_max_tuning_duration(max_tuning_ms)
        tunable.set_max_tuning_iterations(100)
    elif not tunable.read_file(path):
        tunable.enable(False)
        return False
    return True


def flush(path: Optional[str] = None) -> int:
    """Write the current TunableOp table (validators + one row per tuned GEMM) to ``path``;
    returns the number of GEMM rows.  Same CSV layout TunableOp itself reads back."""
    tunable = torch.cuda.tunable
    path = path or DEFAULT_TABLE
    os.makedirs(os.path.dirname(path), exist_ok=True)
    rows = tunable.get_results()
    with open(path + ".tmp", "w") as f:
        for k, v in tunable.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for r in rows:
            f.write(",".join(str(x) for x in r) + "\n")
    os.replace(path + ".tmp", path)
    return len(rows)
