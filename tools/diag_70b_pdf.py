"""Debugging aid: the 70B phase's engine (TP=1, one request at a time, 1,024-token prefill
chunks) on the first `n` documents of the fixed multi-page PDF set (after `nref` of the
reference prompts, as the bench phase runs them), with the traceback of any failure
printed (the bench phase reports only the message).  Usage: diag_70b_pdf.py n [nref]."""
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from replisense_rfq_amd.benchmarks.stream import latency_pdf_set, latency_reference
    from replisense_rfq_amd.engine.engine import LLMEngine
    from replisense_rfq_amd.utils.config import EngineConfig

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    nref = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    cfg = EngineConfig.from_env(model="llama3-70b", seed=0, max_num_seqs=8, graph_buckets=(1,),
                                max_batched_tokens=1024, gemm_split=False)
    eng = LLMEngine(cfg)
    from replisense_rfq_amd import ops
    plans = {name: {str(k): v for k, v in getattr(ops, name).items()}
             for name in ("_LINEAR_PLAN", "_SILU_PLAN", "_NORM_PLAN", "_ROPE_PLAN", "_SWI_PLAN")
             if isinstance(getattr(ops, name, None), dict)}
    print("engine up; small-M plans", json.dumps(plans), "tuned", ops._TUNED_MS, flush=True)
    try:
        if nref:
            lat, _, _ = latency_reference(eng, nref)
            print("reference set", lat, flush=True)
        res = latency_pdf_set(eng, n)
        print(json.dumps(res)[:3000], flush=True)
    except Exception:  # noqa: BLE001 -- the point of the tool
        traceback.print_exc()
        sys.exit(1)


if __name__ == "__main__":
    main()
