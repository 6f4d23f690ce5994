"""The bench's 70B TP=1 latency phase on its own (benchmarks.phases.model_phase), for
A/B runs of the decode weight layout (RFQ_TILED_WEIGHTS=auto|0).  Prints one JSON line."""
import json
import logging
import sys

sys.path.insert(0, ".")
from replisense_rfq_amd.benchmarks.phases import model_phase  # noqa: E402

if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO)
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    print(json.dumps(model_phase("llama3-70b", seed=0, latency_runs=runs, budget_s=400,
                                 in_flight=8)), flush=True)
