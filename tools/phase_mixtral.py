"""The bench's Mixtral 8x7B phase on its own (benchmarks.phases.model_phase with the
driver's settings: 768 in flight, mixed PDF / XLSX uploads, BASELINE config 5), for a
rocprofv3 step window.  Prints one JSON line.

  python tools/phase_mixtral.py [docs] [warm]
"""
import json
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd.benchmarks.phases import model_phase  # noqa: E402

if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO)
    docs = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    print(json.dumps(model_phase("mixtral-8x7b", seed=0, in_flight=768, warm_docs=warm,
                                 docs=docs, formats=("pdf", "xlsx"), budget_s=400,
                                 max_batched_tokens=16384)), flush=True)
