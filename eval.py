"""HellaSwag evaluation CLI (reference eval.py): `python eval.py -m custom -d cuda`.

Same flags as the reference (-m/--model_type, -v/--hf_model_name, -d/--device) plus
--checkpoint, --data-dir, --num-examples, --out-file, --dtype.  Implementation:
mamba_distributed_amd/evaluation/hellaswag.py.
"""
from mamba_distributed_amd.evaluation.hellaswag import (ModelType, evaluate, iterate_examples,  # noqa: F401
                                                        load_model_from_checkpoint, main, render_example)

if __name__ == "__main__":
    main()
