"""The bench's Llama-3-70B phase alone (TP=1, one request at a time): the reference's 14
recorded prompts and the fixed multi-page PDF set (BASELINE config 4).  Prints the phase
JSON.  Usage: phase_70b_pdf.py [latency_runs] [pdf_set]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from replisense_rfq_amd.benchmarks import phases as ph

    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    pdf = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    res = ph.model_phase("llama3-70b", seed=0, latency_runs=runs, budget_s=400.0, in_flight=8,
                         reference_set=True, pdf_set=pdf, graph_buckets=(1,),
                         max_batched_tokens=1024, gemm_split=False)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
