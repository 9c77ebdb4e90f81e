"""The f3 validation bench (validate_bench.run_validate_bench: ResNet-18 W2A4, batch 128,
3 warm-up + 20 timed batches) for a rocprofv3 kernel trace; tools/val_summary.py groups
the trace's launches per validation batch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shiftedscalequantization_amd.validate_bench import run_validate_bench  # noqa: E402

r = run_validate_bench(torch.device("cuda"), 1, 0)
r.pop("_elapsed_s")
print(json.dumps(r), flush=True)
