// pybind11 bindings of the host runtime: replisense_rfq_amd._runtime
#include <cstring>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_manager.h"
#include "engine_core.h"
#include "grammar.h"
#include "shm_ring.h"

namespace py = pybind11;
using namespace rfqrt;

template <typename T>
using arr = py::array_t<T, py::array::c_style | py::array::forcecast>;

template <typename T>
static std::vector<T> vec(const py::dict& d, const char* k) {
  arr<T> a = d[k].cast<arr<T>>();
  return std::vector<T>(a.data(), a.data() + a.size());
}

static Grammar* make_grammar(const py::dict& d) {
  auto* g = new Grammar();
  auto ops = vec<int32_t>(d, "ops");
  for (size_t i = 0; i + 6 <= ops.size(); i += 6)
    g->ops.push_back(Op{ops[i], ops[i + 1], ops[i + 2], ops[i + 3], ops[i + 4], ops[i + 5]});
  g->lit_off = vec<int32_t>(d, "lit_off");
  g->lit_tok = vec<int32_t>(d, "lit_tok");
  g->lit1_off = vec<int32_t>(d, "lit1_off");
  g->lit1_tok = vec<int32_t>(d, "lit1_tok");
  g->lit_first = vec<int32_t>(d, "lit_first");
  g->choice_off = vec<int32_t>(d, "choice_off");
  auto alts = vec<int32_t>(d, "alts");
  for (size_t i = 0; i + 6 <= alts.size(); i += 6)
    g->alts.push_back(Alt{alts[i], alts[i + 1], alts[i + 2], alts[i + 3], alts[i + 4], alts[i + 5]});
  g->alt_rest = vec<int32_t>(d, "alt_rest");
  g->choice_masks = vec<int32_t>(d, "choice_masks");
  g->max_items = vec<int32_t>(d, "max_items");
  g->honors_min = vec<int32_t>(d, "honors_min");
  g->caps = vec<int32_t>(d, "caps");
  g->num_masks = vec<int32_t>(d, "num_masks");
  g->num_caps = vec<int32_t>(d, "num_caps");
  g->fin = vec<int32_t>(d, "fin");
  g->fin1 = vec<int32_t>(d, "fin1");
  g->close_alt = vec<int32_t>(d, "close_alt");
  g->null_ids = vec<int32_t>(d, "null_ids");
  g->tok_class = vec<uint8_t>(d, "tok_class");
  g->tok_chars = vec<uint8_t>(d, "tok_chars");
  g->tok_digits = vec<uint8_t>(d, "tok_digits");
  g->tok_utf = vec<uint8_t>(d, "tok_utf");
  auto sm = vec<int32_t>(d, "str_masks");
  if (sm.size() != STR_SUBS) throw py::value_error("str_masks must hold 5 rows");
  std::copy(sm.begin(), sm.end(), g->str_masks);
  // quote zero dot backslash slack start ncap cont
  auto sc = vec<int32_t>(d, "scalars");
  g->quote = sc[0]; g->zero = sc[1]; g->dot = sc[2]; g->backslash = sc[3]; g->slack = sc[4];
  g->start_pc = sc[5]; g->ncap = sc[6]; g->cont = sc[7];
  const size_t nops = g->ops.size(), nch = g->choice_off.size() - 1;
  if (g->fin.size() != nops * NPROF || g->fin1.size() != nops * NPROF ||
      g->close_alt.size() != nch * NPROF || g->choice_masks.size() != nch * 8 ||
      g->caps.size() != (size_t)g->ncap * NPROF || g->null_ids.empty() ||
      g->tok_utf.size() != g->tok_class.size() ||
      g->num_caps.size() * NUM_PHASES != g->num_masks.size() * 2)
    throw py::value_error("inconsistent grammar tables");
  return g;
}

static py::tuple state_tuple(const State& s) {
  return py::make_tuple(s.pc, s.sub, s.cnt, s.rem, s.minv, s.prof);
}

static State state_of(const py::tuple& st) {
  if (st.size() != 6) throw py::value_error("grammar state must have 6 fields");
  return State{st[0].cast<int32_t>(), st[1].cast<int32_t>(), st[2].cast<int32_t>(),
               st[3].cast<int32_t>(), st[4].cast<int32_t>(), st[5].cast<int32_t>()};
}

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "replisense_rfq_amd native host runtime (grammar automaton, KV block manager)";

  py::class_<Grammar, std::shared_ptr<Grammar>>(m, "Grammar")
      .def(py::init(&make_grammar))
      .def("initial", [](const Grammar& g, int32_t min_items, int32_t profile, int32_t budget) {
        std::vector<int32_t> forced;
        State s = g.initial(forced, min_items, profile, budget);
        return py::make_tuple(state_tuple(s), forced);
      }, py::arg("min_items") = 0, py::arg("profile") = 0, py::arg("budget") = NO_BUDGET)
      .def("advance", [](const Grammar& g, py::tuple st, int32_t tok, int32_t budget) {
        State s = state_of(st);
        std::vector<int32_t> forced;
        if (!g.advance(s, tok, forced, budget)) throw py::value_error("token not allowed by grammar");
        return py::make_tuple(state_tuple(s), forced);
      }, py::arg("state"), py::arg("token"), py::arg("budget") = NO_BUDGET)
      .def("mask", [](const Grammar& g, py::tuple st) { return g.mask(state_of(st)); })
      .def("close_cost", [](const Grammar& g, py::tuple st) { return g.close_cost(state_of(st)); })
      // states: int32 [n, 6] updated in place; tokens, budgets: int32 [n]
      // returns (mask_idx[n] (-1 = finished), forced_offsets[n+1], forced_tokens, ok[n])
      .def("batch_advance", [](const Grammar& g, py::array_t<int32_t, py::array::c_style> states,
                               arr<int32_t> tokens, arr<int32_t> budgets) {
        const py::ssize_t n = tokens.size();
        if (states.ndim() != 2 || states.shape(0) != n || states.shape(1) != 6)
          throw py::value_error("states must be int32 [n, 6]");
        if (budgets.size() != n) throw py::value_error("budgets must be int32 [n]");
        auto S = states.mutable_unchecked<2>();
        const int32_t* tk = tokens.data();
        const int32_t* bg = budgets.data();
        py::array_t<int32_t> masks(n), offs(n + 1);
        py::array_t<bool> ok(n);
        auto M = masks.mutable_unchecked<1>();
        auto O = offs.mutable_unchecked<1>();
        auto K = ok.mutable_unchecked<1>();
        std::vector<int32_t> forced;
        forced.reserve(n * 8);
        {
          py::gil_scoped_release nogil;
          for (py::ssize_t i = 0; i < n; ++i) {
            O(i) = (int32_t)forced.size();
            State s{S(i, 0), S(i, 1), S(i, 2), S(i, 3), S(i, 4), S(i, 5)};
            const bool good = g.advance(s, tk[i], forced, bg[i]);
            K(i) = good;
            S(i, 0) = s.pc; S(i, 1) = s.sub; S(i, 2) = s.cnt; S(i, 3) = s.rem; S(i, 4) = s.minv;
            S(i, 5) = s.prof;
            M(i) = g.mask(s);
          }
          O(n) = (int32_t)forced.size();
        }
        py::array_t<int32_t> ft(forced.size());
        std::copy(forced.begin(), forced.end(), ft.mutable_data());
        return py::make_tuple(masks, offs, ft, ok);
      })
      .def_readonly("slack", &Grammar::slack)
      .def("num_ops", [](const Grammar& g) { return (int)g.ops.size(); });

  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int32_t, int32_t>())
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("num_free", &BlockManager::num_free)
      .def_property_readonly("num_cached", &BlockManager::num_cached)
      .def_readonly("hits", &BlockManager::hits)
      .def_readonly("queries", &BlockManager::queries)
      .def_readonly("evictions", &BlockManager::evictions)
      .def("allocate", [](BlockManager& bm, int32_t n) -> py::object {
        std::vector<int32_t> out;
        if (!bm.allocate(n, out)) return py::none();
        return py::cast(out);
      })
      .def("release", [](BlockManager& bm, const std::vector<int32_t>& blocks) {
        bm.release(blocks.data(), (int32_t)blocks.size());
      })
      .def("match_prefix", [](BlockManager& bm, const std::vector<uint64_t>& hashes) {
        std::vector<int32_t> out;
        bm.match_prefix(hashes.data(), (int32_t)hashes.size(), out);
        return out;
      })
      .def("register_block", &BlockManager::register_block)
      .def("refcount", &BlockManager::refcount)
      .def_static("hash_blocks", [](arr<int32_t> tokens, int32_t block_size, uint64_t parent) {
        const int32_t n = (int32_t)tokens.size() / block_size;
        std::vector<uint64_t> out(n);
        const int32_t* t = tokens.data();
        for (int32_t i = 0; i < n; ++i) {
          parent = BlockManager::hash_block(parent, t + (int64_t)i * block_size, block_size);
          out[i] = parent;
        }
        return out;
      }, py::arg("tokens"), py::arg("block_size"), py::arg("parent") = 0);

  py::class_<EngineCore>(m, "EngineCore")
      .def(py::init([](const py::dict& c, std::shared_ptr<Grammar> g) {
             CoreConfig cfg;
             auto geti = [&](const char* k, int32_t& v) { if (c.contains(k)) v = c[k].cast<int32_t>(); };
             auto getb = [&](const char* k, bool& v) { if (c.contains(k)) v = c[k].cast<bool>(); };
             geti("block_size", cfg.block_size);
             geti("num_blocks", cfg.num_blocks);
             geti("scratch_block", cfg.scratch_block);
             geti("max_num_seqs", cfg.max_num_seqs);
             geti("max_batched_tokens", cfg.max_batched_tokens);
             geti("max_model_len", cfg.max_model_len);
             geti("ext_max", cfg.ext_max);
             geti("group", cfg.group);
             geti("hkv", cfg.hkv);
             geti("decode_tiles", cfg.decode_tiles);
             geti("prefill_qblk", cfg.prefill_qblk);
             if (cfg.prefill_qblk != 32 && cfg.prefill_qblk != 64)
               throw py::value_error("prefill_qblk must be 32 or 64");
             getb("jump_forward", cfg.jump_forward);
             getb("prefix_cache", cfg.prefix_cache);
             getb("is_cuda", cfg.is_cuda);
             getb("use_graphs", cfg.use_graphs);
             if (c.contains("token_mults")) cfg.token_mults = c["token_mults"].cast<std::vector<int32_t>>();
             if (c.contains("eos_ids")) cfg.eos_ids = c["eos_ids"].cast<std::vector<int32_t>>();
             if (cfg.num_blocks <= 0) throw py::value_error("num_blocks must be > 0");
             return new EngineCore(cfg, std::const_pointer_cast<const Grammar>(g));
           }), py::arg("config"), py::arg("grammar") = nullptr)
      .def("add", [](EngineCore& e, arr<int32_t> prompt, float temperature, int32_t max_tokens,
                     int64_t seed, bool grammar, int32_t min_items, int32_t profile,
                     double t_arrival) {
        SeqParams p{temperature, max_tokens, seed, grammar, min_items, profile};
        return e.add(prompt.data(), (int32_t)prompt.size(), p, t_arrival);
      })
      .def("schedule_and_pack", [](EngineCore& e, py::array_t<int32_t, py::array::c_style> header,
                                   py::array_t<int32_t, py::array::c_style> payload, double now) {
        if (header.size() < HEADER) throw py::value_error("header must hold 16 int32");
        if (reinterpret_cast<uintptr_t>(payload.data()) % 8)
          throw py::value_error("payload must be 8-byte aligned");
        int32_t* h = header.mutable_data();
        int32_t* p = payload.mutable_data();
        const int64_t cap = payload.size();
        py::gil_scoped_release nogil;
        return e.schedule_and_pack(h, p, cap, now);
      })
      .def("post", [](EngineCore& e, arr<int32_t> sampled, double now) {
        const int32_t* t = sampled.data();
        const int32_t n = (int32_t)sampled.size();
        py::gil_scoped_release nogil;
        return e.post(t, n, now);
      })
      .def("abort_all", [](EngineCore& e, int reason, double now) {
        return e.abort_all((FinishReason)reason, now);
      })
      .def("drain_finished", &EngineCore::drain_finished)
      .def("abort", [](EngineCore& e, int32_t id, int reason, double now) {
        return e.abort(id, (FinishReason)reason, now);
      })
      .def("release", &EngineCore::release)
      .def("set_graph_keys", &EngineCore::set_graph_keys)
      .def("set_max_batched_tokens", &EngineCore::set_max_batched_tokens)
      .def_property_readonly("max_batched_tokens",
                             [](const EngineCore& e) { return e.cfg().max_batched_tokens; })
      .def("graph_key", &EngineCore::find_graph_key)
      .def("pin_prefix", [](EngineCore& e, arr<int32_t> tokens) {
        return e.pin_prefix(tokens.data(), (int32_t)tokens.size());
      })
      .def_property_readonly("num_pinned", &EngineCore::num_pinned)
      .def("payload_bound", &EngineCore::payload_bound)
      .def("tokens", [](const EngineCore& e, int32_t id) {
        const Seq& s = e.seq(id);
        py::array_t<int32_t> out(s.tokens.size());
        std::copy(s.tokens.begin(), s.tokens.end(), out.mutable_data());
        return out;
      })
      .def("info", [](const EngineCore& e, int32_t id) {
        const Seq& s = e.seq(id);
        py::dict d;
        d["prompt_len"] = s.prompt_len;
        d["num_tokens"] = (int32_t)s.tokens.size();
        d["num_cached"] = s.num_cached;
        d["prefix_hit"] = s.prefix_hit;
        d["num_sampled"] = s.num_sampled;
        d["num_forced"] = s.num_forced;
        d["num_blocks"] = (int32_t)s.blocks.size();
        d["status"] = (int)s.status;
        d["finish"] = (int)s.finish;
        d["mask_idx"] = s.mask_idx;
        d["t_first_sched"] = s.t_first_sched;
        d["t_prefill_done"] = s.t_prefill_done;
        d["t_first_token"] = s.t_first_token;
        d["t_finish"] = s.t_finish;
        return d;
      })
      .def_property_readonly("has_work", &EngineCore::has_work)
      .def_property_readonly("num_running", &EngineCore::num_running)
      .def_property_readonly("num_waiting", &EngineCore::num_waiting)
      .def_readonly("num_preempted", &EngineCore::num_preempted)
      .def_readonly("num_steps", &EngineCore::num_steps)
      .def_property_readonly("num_free_blocks", [](EngineCore& e) { return e.bm().num_free(); })
      .def_property_readonly("num_cached_blocks", [](EngineCore& e) { return e.bm().num_cached(); })
      .def_property_readonly("prefix_hits", [](EngineCore& e) { return e.bm().hits; })
      .def_property_readonly("prefix_queries", [](EngineCore& e) { return e.bm().queries; })
      .def_property_readonly("evictions", [](EngineCore& e) { return e.bm().evictions; });

  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, int64_t, int, bool, int>(), py::arg("name"),
           py::arg("capacity"), py::arg("n_readers"), py::arg("create"), py::arg("reader_id") = -1)
      .def("publish", [](ShmRing& r, py::array_t<int32_t, py::array::c_style> msg, double timeout) {
        const void* p = msg.data();
        const int64_t n = (int64_t)msg.size() * 4;
        py::gil_scoped_release nogil;
        return r.publish(p, n, timeout);
      })
      .def("receive", [](ShmRing& r, double timeout) -> py::object {
        std::vector<uint8_t> buf;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = r.receive(buf, timeout);
        }
        if (!ok) return py::none();
        py::array_t<int32_t> out((py::ssize_t)(buf.size() / 4));
        std::memcpy(out.mutable_data(), buf.data(), buf.size());
        return out;
      })
      .def_property_readonly("capacity", &ShmRing::capacity)
      .def_property_readonly("name", &ShmRing::name);
}
