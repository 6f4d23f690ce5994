"""replisense_rfq_amd — MI355X-native RFQ extraction service.

Layers:
  api/       FastAPI surface, byte-compatible with the reference app/main.py
  service/   document ingestion (CPU) + extraction service (prompt, schema, recovery)
  engine/    on-node LLM inference engine: scheduler, paged KV, prefix cache,
             JSON-schema grammar, tokenizer, hipGraph decode, DP router
  models/    Llama-3 (8B/70B) and Mixtral-8x7B on the gfx950 kernels
  ops/       dispatch to the hand-written HIP kernels (csrc/kernels) + torch oracles
  parallel/  tensor parallelism over RCCL/xGMI, process groups, control plane
  runtime/   C++ runtime bindings (block allocator, grammar automaton)
  utils/     config, logging, tracing
"""
__version__ = "2.0.0"
