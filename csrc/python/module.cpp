// xflow-amd: Python bindings (pybind11) of the native core.
//
// Device buffers cross the boundary as integer addresses (torch's
// tensor.data_ptr()) so the module has no libtorch dependency; the Python
// layer (xflow_amd/engine.py) owns shape/dtype/device checks.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#include <string>

#include "../comm/async_ps.h"
#include "../comm/rccl_comm.h"
#include "../comm/sharded_step.h"
#include "xflow/engine.h"
#include "xflow/reader.h"
#include "xflow/trainer.h"

namespace py = pybind11;
using namespace xflow;

namespace {

template <typename T>
T* P(uintptr_t a) {
  return reinterpret_cast<T*>(a);
}

template <typename T>
py::array_t<T> to_np(const std::vector<T>& v) {
  py::array_t<T> a((py::ssize_t)v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), sizeof(T) * v.size());
  return a;
}

py::dict block_to_dict(const CsrBlock& b) {
  py::dict d;
  d["row_ptr"] = to_np(b.row_ptr);
  d["keys"] = to_np(b.keys);
  d["fgid"] = to_np(b.fgid);
  d["labels"] = to_np(b.labels);
  d["max_fgid"] = b.max_fgid;
  return d;
}

py::dict stats_dict(const LossStats& s) {
  py::dict d;
  d["ln_loss"] = s.ln_loss;
  d["log2_lik"] = s.log2_lik;
  d["rows"] = s.rows;
  d["positives"] = s.positives;
  return d;
}

ModelSpec model_from(py::dict d) {
  ModelSpec m;
  if (d.contains("kind")) m.kind = d["kind"].cast<int>();
  if (d.contains("v_dim")) m.v_dim = d["v_dim"].cast<int>();
  if (d.contains("fm_math")) m.fm_math = d["fm_math"].cast<int>();
  if (d.contains("mvm_math")) m.mvm_math = d["mvm_math"].cast<int>();
  if (d.contains("fm_mfma")) m.fm_mfma = d["fm_mfma"].cast<bool>() ? 1 : 0;
  return m;
}

OptSpec opt_from(py::dict d) {
  OptSpec o;
  if (d.contains("kind")) o.kind = d["kind"].cast<int>();
  if (d.contains("alpha")) o.ftrl.alpha = d["alpha"].cast<float>();
  if (d.contains("beta")) o.ftrl.beta = d["beta"].cast<float>();
  if (d.contains("lambda1")) o.ftrl.lambda1 = d["lambda1"].cast<float>();
  if (d.contains("lambda2")) o.ftrl.lambda2 = d["lambda2"].cast<float>();
  if (d.contains("lr")) o.sgd.lr = d["lr"].cast<float>();
  if (d.contains("sgd_v_init")) o.sgd.v_init = d["sgd_v_init"].cast<float>();
  if (d.contains("v_init_scale")) o.v_init_scale = d["v_init_scale"].cast<float>();
  if (d.contains("seed")) o.seed = d["seed"].cast<uint64_t>();
  return o;
}

py::dict plan_dict(const StepPlan& p) {
  py::dict d;
  d["S"] = p.S;
  d["groups"] = p.groups;
  d["Sf"] = p.Sf;
  d["csr_slog2"] = p.csr_slog2;
  d["csr_rows"] = p.csr_rows;
  d["grad"] = grad_path_name(p.grad);
  d["masks"] = p.masks;
  d["upos"] = p.upos;
  d["lr16"] = p.lr16;
  d["lr16s"] = p.lr16s;
  d["uqm"] = p.uqm;
  d["fmu"] = p.fmu;
  d["fm_keep_w"] = p.fm_keep_w;
  d["mvmu"] = p.mvmu;
  d["fsu"] = p.fsu;
  d["rowu"] = p.rowu;
  d["grpst"] = p.grpst;
  d["uq"] = p.uq;
  return d;
}

// {model, opt, gpu, remaps, red_pairs, red_rowv, fm_vals, csr, sum_slices,
//  scratch_cap, max_nnz, slice_cap}; the table layout and pstride follow
// from model and opt
StepInputs inputs_from(py::dict d) {
  StepInputs in;
  const ModelSpec m = model_from(d["model"].cast<py::dict>());
  const OptSpec o = opt_from(d["opt"].cast<py::dict>());
  in.kind = m.kind;
  in.fm_math = m.fm_math;
  in.L = TableLayout::make(m, o);
  in.pstride = m.pstride();
  auto flag = [&](const char* k, bool def) { return d.contains(k) ? d[k].cast<bool>() : def; };
  in.gpu = flag("gpu", true);
  in.remaps = flag("remaps", in.gpu);
  in.red_pairs = flag("red_pairs", in.gpu);
  in.red_rowv = flag("red_rowv", in.gpu && (m.kind == kMVM || (m.kind == kFM && m.fm_math == kFmStandard)));
  in.fm_vals = flag("fm_vals", in.gpu && m.kind == kFM && m.fm_math == kFmReference);
  in.csr = flag("csr", true);
  in.sum_slices = flag("sum_slices", false);
  in.max_nnz = d.contains("max_nnz") ? d["max_nnz"].cast<double>() : (double)(1 << 22);
  in.scratch_cap = d.contains("scratch_cap") ? d["scratch_cap"].cast<double>() : 4.0 * in.max_nnz;
  in.slice_cap = d.contains("slice_cap") ? d["slice_cap"].cast<int>() : Engine::kSliceGroup;
  in.max_rows = d.contains("max_rows") ? d["max_rows"].cast<double>() : (double)(1 << 16);
  in.kdim = m.kernel_dim();
  return in;
}

}  // namespace

PYBIND11_MODULE(_xflow_native, m) {
  m.doc() = "xflow-amd native core: HBM hash-table engine, gfx950 kernels, libffm reader";

  m.def("hip_available", &hip_backend_available);
  // the single-rank step's layout decisions for hypothetical inputs (tests)
  m.def("plan_step", [](py::dict inputs, int S) { return plan_dict(plan_step(inputs_from(inputs), S)); });
  // The reference's pred_<rank>_<block>.txt (lr_worker.cc:65-68: `pctr \t
  // 1-label \t label`, ostream default float format = %g): formatted into one
  // buffer and written with a single fwrite, without the GIL.
  m.def("write_pred", [](const std::string& path, py::array_t<float> pctr,
                         py::array_t<int32_t> labels) {
    const int64_t n = pctr.size();
    if (labels.size() != n) throw std::invalid_argument("write_pred: lengths differ");
    const float* p = pctr.data();
    const int32_t* y = labels.data();
    py::gil_scoped_release nogil;
    // chunks formatted in parallel (std::to_chars general/6 == printf "%g")
    const int64_t per = 1 << 18;
    const int64_t nchunk = (n + per - 1) / per;
    std::vector<std::string> out((size_t)nchunk);
    std::atomic<int64_t> next{0};
    auto work = [&]() {
      for (int64_t c = next++; c < nchunk; c = next++) {
        const int64_t lo = c * per, hi = lo + per < n ? lo + per : n;
        std::string& b = out[(size_t)c];
        b.resize((size_t)(hi - lo) * 24);
        char* q = &b[0];
        for (int64_t i = lo; i < hi; ++i) {
          q = std::to_chars(q, q + 16, (double)p[i], std::chars_format::general, 6).ptr;
          const int yi = y[i] ? 1 : 0;
          *q++ = '\t';
          *q++ = (char)('0' + (1 - yi));
          *q++ = '\t';
          *q++ = (char)('0' + yi);
          *q++ = '\n';
        }
        b.resize((size_t)(q - &b[0]));
      }
    };
    const unsigned hw = std::thread::hardware_concurrency();
    const int nt = (int)std::min<int64_t>(nchunk, hw ? (hw < 16 ? hw : 16) : 4);
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (std::thread& t : th) t.join();
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("write_pred: cannot open " + path);
    bool ok = true;
    for (const std::string& b : out) ok = ok && std::fwrite(b.data(), 1, b.size(), f) == b.size();
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) throw std::runtime_error("write_pred: write failed " + path);
  });
  m.def("feature_hash", [](py::bytes b) {
    std::string s = b;
    return feature_hash(s.data(), s.size());
  });
  m.def("parse_libffm", [](py::bytes b) {
    std::string s = b;
    CsrBlock blk;
    parse_libffm(s.data(), s.size(), blk);
    return block_to_dict(blk);
  });
  m.def("reference_auc", [](py::array_t<int32_t> labels, py::array_t<float> pctr) {
    auto l = labels.unchecked<1>();
    auto p = pctr.unchecked<1>();
    std::vector<std::pair<int, float>> v;
    for (py::ssize_t i = 0; i < l.shape(0); ++i) v.emplace_back(l(i), p(i));
    EvalResult r = reference_auc(v);
    py::dict d;
    d["logloss_printed"] = r.logloss_printed;
    d["ln_logloss"] = r.ln_logloss;
    d["auc"] = r.auc;
    d["tp"] = r.tp;
    d["n"] = r.n;
    d["line"] = r.line;
    return d;
  });

  py::class_<BatchView>(m, "BatchView")
      .def(py::init<>())
      .def_property("keys", [](const BatchView& b) { return (uintptr_t)b.keys; },
                    [](BatchView& b, uintptr_t v) { b.keys = P<const u64>(v); })
      .def_property("row_ptr", [](const BatchView& b) { return (uintptr_t)b.row_ptr; },
                    [](BatchView& b, uintptr_t v) { b.row_ptr = P<const int32_t>(v); })
      .def_property("fgid", [](const BatchView& b) { return (uintptr_t)b.fgid; },
                    [](BatchView& b, uintptr_t v) { b.fgid = P<const int32_t>(v); })
      .def_property("labels", [](const BatchView& b) { return (uintptr_t)b.labels; },
                    [](BatchView& b, uintptr_t v) { b.labels = P<const float>(v); })
      .def_readwrite("rows", &BatchView::rows)
      .def_readwrite("nnz", &BatchView::nnz)
      .def_readwrite("nnz_per_row", &BatchView::nnz_per_row)
      .def_readwrite("slice_rows", &BatchView::slice_rows)
      .def_readwrite("col_stride", &BatchView::col_stride);

  py::class_<RcclComm>(m, "RcclComm")
      .def_static("unique_id",
                  []() {
                    auto v = RcclComm::unique_id();
                    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
                  })
      .def(py::init([](py::bytes id, int world, int rank, int device) {
             std::string s = id;
             std::vector<uint8_t> v(s.begin(), s.end());
             py::gil_scoped_release nogil;  // blocks until every rank joined
             return new RcclComm(v, world, rank, device);
           }),
           py::arg("id"), py::arg("world"), py::arg("rank"), py::arg("device"))
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("rank", &RcclComm::rank)
      .def("alltoallv",
           [](RcclComm& c, uintptr_t send, std::vector<int64_t> sc, uintptr_t recv,
              std::vector<int64_t> rc, int elem_bytes, uintptr_t stream) {
             c.alltoallv(P<const void>(send), sc, P<void>(recv), rc, elem_bytes, stream);
           })
      .def("alltoall",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, int64_t count, int elem_bytes,
              uintptr_t stream) { c.alltoall(P<const void>(send), P<void>(recv), count,
                                             elem_bytes, stream); })
      .def("alltoallv_group",
           [](RcclComm& c, std::vector<uintptr_t> sends, std::vector<uintptr_t> recvs,
              std::vector<int> elem_bytes, std::vector<std::vector<int64_t>> sc,
              std::vector<std::vector<int64_t>> rc, uintptr_t stream) {
             std::vector<RcclComm::A2AOp> ops;
             const size_t n = sends.size();
             if (recvs.size() != n || elem_bytes.size() != n || sc.size() != n || rc.size() != n)
               throw std::invalid_argument("alltoallv_group: list lengths differ");
             for (size_t i = 0; i < n; ++i)
               ops.push_back({P<const void>(sends[i]), sc[i], P<void>(recvs[i]), rc[i],
                              elem_bytes[i]});
             c.alltoallv_group(ops, stream);
           })
      .def("send_recv",
           [](RcclComm& c, std::vector<int> peers, std::vector<uintptr_t> sends,
              std::vector<int64_t> send_bytes, std::vector<uintptr_t> recvs,
              std::vector<int64_t> recv_bytes, uintptr_t stream) {
             c.send_recv(peers, sends, send_bytes, recvs, recv_bytes, stream);
           })
      .def("abort", &RcclComm::abort);

  py::class_<ShardedStep>(m, "ShardedStep")
      .def(py::init([](Engine& e, RcclComm* comm, int world, int rank, bool early_keys,
                       int staleness) {
             return new ShardedStep(e, comm, world, rank, early_keys, staleness);
           }),
           py::arg("engine"), py::arg("comm"), py::arg("world"), py::arg("rank"),
           py::arg("early_keys") = true, py::arg("staleness") = 0, py::keep_alive<1, 2>(),
           py::keep_alive<1, 3>())
      .def("flush", &ShardedStep::flush, py::call_guard<py::gil_scoped_release>())
      .def_readwrite("p2p_ops", &ShardedStep::p2p_ops)
      .def("train_step",
           [](ShardedStep& s, const BatchView& b, int64_t id, int S, py::object next,
              int64_t next_id, py::object prefetch) {
             BatchView nv;
             const bool has = !next.is_none();
             if (has) nv = next.cast<BatchView>();
             std::function<void()> pf;
             if (!prefetch.is_none()) {
               pf = [prefetch]() {
                 py::gil_scoped_acquire gil;
                 prefetch();
               };
             }
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = s.train_step(b, id, S, has ? &nv : nullptr, next_id, pf);
             }
             return ok;
           },
           py::arg("batch"), py::arg("id"), py::arg("S"), py::arg("next") = py::none(),
           py::arg("next_id") = 0, py::arg("prefetch") = py::none())
      .def("eval_step",
           [](ShardedStep& s, const BatchView& b, uintptr_t pctr) {
             return s.eval_step(b, P<float>(pctr));
           },
           py::call_guard<py::gil_scoped_release>())
      .def_readwrite("host_waits", &ShardedStep::host_waits)
      .def_readwrite("mid_step_waits", &ShardedStep::mid_step_waits)
      .def_readwrite("buffer_growths", &ShardedStep::buffer_growths)
      .def_readwrite("csr_exchanges", &ShardedStep::csr_exchanges)
      .def_readwrite("csr_waits", &ShardedStep::csr_waits)
      .def_readwrite("csr_wait_s", &ShardedStep::csr_wait_s)
      .def_readwrite("early_key_exchanges", &ShardedStep::early_key_exchanges)
      .def_readwrite("inline_prepares", &ShardedStep::inline_prepares)
      .def_readwrite("empty_steps", &ShardedStep::empty_steps)
      .def_readwrite("bytes_moved", &ShardedStep::bytes_moved)
      .def_readwrite("drop_exchanges", &ShardedStep::drop_exchanges)
      .def_readwrite("host_wait_s", &ShardedStep::host_wait_s)
      .def_readonly("last_send", &ShardedStep::last_send)
      .def_readonly("last_recv", &ShardedStep::last_recv);

  py::class_<AsyncPS>(m, "AsyncPS")
      .def(py::init([](Engine& worker, Engine& server, int world, int rank, int staleness,
                       int slices, std::string name, double timeout_s, int slow_ms,
                       double pair_frac, int device) {
             AsyncPS::Config c;
             c.world = world;
             c.rank = rank;
             c.staleness = staleness;
             c.slices = slices;
             c.name = name;
             c.timeout_s = timeout_s;
             c.slow_ms = slow_ms;
             c.pair_frac = pair_frac;
             c.device = device;
             return new AsyncPS(worker, server, c);
           }),
           py::arg("worker"), py::arg("server"), py::arg("world"), py::arg("rank"),
           py::arg("staleness"), py::arg("slices"), py::arg("name"), py::arg("timeout_s") = 600.0,
           py::arg("slow_ms") = 0, py::arg("pair_frac") = 1.0, py::arg("device") = -1,
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def("handle",
           [](const AsyncPS& a) {
             auto v = a.handle();
             return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
           })
      .def("connect",
           [](AsyncPS& a, std::vector<py::bytes> hs) {
             std::vector<std::vector<uint8_t>> v;
             for (auto& h : hs) {
               std::string s = h;
               v.emplace_back(s.begin(), s.end());
             }
             a.connect(v);
           })
      .def("start", &AsyncPS::start)
      .def("train_step", &AsyncPS::train_step, py::call_guard<py::gil_scoped_release>())
      .def("eval_step",
           [](AsyncPS& a, const BatchView& b, uintptr_t pctr) { return a.eval_step(b, P<float>(pctr)); },
           py::call_guard<py::gil_scoped_release>())
      .def("finish", &AsyncPS::finish, py::call_guard<py::gil_scoped_release>())
      .def("stop", &AsyncPS::stop, py::call_guard<py::gil_scoped_release>())
      .def("log", [](const AsyncPS& a) { return to_np(a.log()); })
      .def_property_readonly("serving", &AsyncPS::serving)
      .def_property_readonly("transport", &AsyncPS::transport)
      .def_property_readonly("csr", &AsyncPS::csr)
      .def_readonly("steps", &AsyncPS::steps)
      .def_readonly("evals", &AsyncPS::evals)
      .def_readwrite("bytes_moved", &AsyncPS::bytes_moved)
      .def_readwrite("max_staleness", &AsyncPS::max_staleness)
      .def_readwrite("max_lead", &AsyncPS::max_lead)
      .def_readwrite("wait_slot_s", &AsyncPS::wait_slot_s)
      .def_readwrite("wait_pull_s", &AsyncPS::wait_pull_s)
      .def_readwrite("sync_s", &AsyncPS::sync_s)
      .def_readonly("served_pulls", &AsyncPS::served_pulls)
      .def_readonly("applied_pushes", &AsyncPS::applied_pushes)
      .def_readonly("server_busy_s", &AsyncPS::server_busy_s);

  py::class_<Engine>(m, "Engine")
      .def(py::init([](py::dict model, py::dict opt, int table_log2_cap, int64_t max_rows,
                       int64_t max_nnz, int max_slices, bool sum_slices, double scratch_factor,
                       int device, bool table_grow, double grow_load, int max_log2_cap,
                       int monitor_lag, int owner_group, double grow_start, bool csr) {
             EngineConfig c;
             c.owner_group = owner_group;
             c.csr = csr;
             c.table_grow = table_grow;
             c.grow_load = grow_load;
             c.grow_start = grow_start;
             c.max_log2_cap = max_log2_cap;
             c.monitor_lag = monitor_lag;
             c.model = model_from(model);
             c.opt = opt_from(opt);
             c.table_log2_cap = table_log2_cap;
             c.max_rows = max_rows;
             c.max_nnz = max_nnz;
             c.max_slices = max_slices;
             c.sum_slices = sum_slices;
             c.scratch_factor = scratch_factor;
             c.device = device;
             return new Engine(c);
           }),
           py::arg("model"), py::arg("opt"), py::arg("table_log2_cap") = 20,
           py::arg("max_rows") = 1 << 16, py::arg("max_nnz") = 1 << 22,
           py::arg("max_slices") = 1, py::arg("sum_slices") = false,
           py::arg("scratch_factor") = 2.5, py::arg("device") = -1,
           py::arg("table_grow") = true, py::arg("grow_load") = 0.8, py::arg("max_log2_cap") = 0,
           py::arg("monitor_lag") = 2, py::arg("owner_group") = 0, py::arg("grow_start") = 0.6,
           py::arg("csr") = true)
      .def_property_readonly("table_growths", &Engine::table_growths)
      .def_property_readonly("csr_steps", &Engine::csr_steps)
      .def("step_plan", [](const Engine& e, int S) { return plan_dict(e.plan(S)); })
      .def_property_readonly("table_splits", &Engine::table_splits)
      .def_property_readonly("table_geometry", &Engine::table_geometry)
      .def_property_readonly("table_committed", &Engine::table_committed)
      .def_property_readonly("grow_seconds", &Engine::grow_seconds)
      .def_property_readonly("monitor_waits", &Engine::monitor_waits)
      .def_property_readonly("monitor_wait_seconds", &Engine::monitor_wait_seconds)
      .def("parse_text",
           [](Engine& e, uintptr_t text, int64_t n, uintptr_t keys, uintptr_t fgid,
              uintptr_t row_ptr, uintptr_t labels, int64_t max_rows, int64_t max_nnz,
              int64_t row_mod) {
             return e.parse_text(P<const char>(text), n, P<u64>(keys), P<int32_t>(fgid),
                                 P<int32_t>(row_ptr), P<float>(labels), max_rows, max_nnz,
                                 row_mod);
           },
           py::arg("text"), py::arg("n"), py::arg("keys"), py::arg("fgid"), py::arg("row_ptr"),
           py::arg("labels"), py::arg("max_rows"), py::arg("max_nnz"), py::arg("row_mod") = 1,
           py::call_guard<py::gil_scoped_release>())
      .def("count_records", &Engine::count_records)
      .def("take_records", &Engine::take_records, py::call_guard<py::gil_scoped_release>())
      .def("grow_table", &Engine::grow_table, py::call_guard<py::gil_scoped_release>())
      .def("end_step", &Engine::end_step, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("is_gpu", &Engine::is_gpu)
      .def_property_readonly("backend_name", [](Engine& e) { return e.backend().name(); })
      .def_property_readonly("pstride", &Engine::pstride)
      .def_property_readonly("grad_width", &Engine::grad_width)
      .def_property_readonly("value_width", &Engine::value_width)
      .def_property_readonly("P", [](Engine& e) { return e.config().model.P(); })
      .def_property_readonly("state_words", &Engine::state_words)
      .def_property_readonly("table_capacity", &Engine::table_capacity)
      .def_property_readonly("table_bytes", &Engine::table_bytes)
      .def_property_readonly("layout", [](Engine& e) {
        const TableLayout& L = e.layout();
        py::dict d;
        d["kind"] = e.config().model.kind;
        d["P"] = L.P;
        d["opt"] = L.opt;
        d["stride"] = L.stride;
        return d;
      })
      .def("set_stream", [](Engine& e, uintptr_t s) { e.set_stream(reinterpret_cast<void*>(s)); })
      .def("synchronize", &Engine::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("train_step", &Engine::train_step, py::call_guard<py::gil_scoped_release>())
      .def("eval_step",
           [](Engine& e, const BatchView& b, uintptr_t pctr) { e.eval_step(b, P<float>(pctr)); },
           py::call_guard<py::gil_scoped_release>())
      .def("slices_of", &Engine::slices_of)
      .def_static("slice_groups", &Engine::slice_groups)
      .def_static("group_slices", &Engine::group_slices)
      .def_readonly_static("slice_group", &Engine::kSliceGroup)
      .def("push_host",
           [](Engine& e, py::array_t<uint64_t> keys, py::array_t<float> grads) {
             std::vector<u64> k(keys.data(), keys.data() + keys.size());
             std::vector<float> g(grads.data(), grads.data() + grads.size());
             e.push_host(k, g);
           })
      .def("eval_metrics",
           [](Engine& e, uintptr_t pctr, uintptr_t labels, int64_t n) {
             EvalMetrics m;
             {
               py::gil_scoped_release nogil;
               m = e.eval_metrics(P<const float>(pctr), P<const float>(labels), n);
             }
             EvalResult r = eval_result(m);
             py::dict d;
             d["n"] = m.n;
             d["tp"] = m.tp;
             d["area"] = m.area;
             d["log2_sum"] = m.log2_sum;
             d["logloss_printed"] = r.logloss_printed;
             d["ln_logloss"] = r.ln_logloss;
             d["auc"] = r.auc;
             d["line"] = r.line;
             return d;
           })
      .def("download_small",
           [](Engine& e, uintptr_t dst, uintptr_t src, size_t bytes) {
             e.download_small(P<void>(dst), P<const void>(src), bytes);
           })
      .def("prefill", &Engine::prefill, py::arg("n"), py::arg("seed") = 0x5eedull,
           py::call_guard<py::gil_scoped_release>())
      .def("pull_host",
           [](Engine& e, py::array_t<uint64_t> keys) {
             std::vector<u64> k(keys.data(), keys.data() + keys.size());
             return to_np(e.pull_host(k));
           })
      .def("w_prepare",
           [](Engine& e, const BatchView& b, int world, uintptr_t counts, uintptr_t send_keys,
              int wb, int64_t seq) {
             e.w_prepare(b, world, P<int64_t>(counts), P<u64>(send_keys), wb, seq);
           },
           py::arg("batch"), py::arg("world"), py::arg("counts"), py::arg("send_keys"),
           py::arg("wb") = 0, py::arg("seq") = -1, py::call_guard<py::gil_scoped_release>())
      .def("s_pull",
           [](Engine& e, uintptr_t keys, int64_t n, uintptr_t out, bool insert, int buf,
              std::vector<int64_t> offsets, bool keep_weights) {
             e.s_pull(P<const u64>(keys), n, P<float>(out), insert, buf, offsets, keep_weights);
           },
           py::arg("keys"), py::arg("n"), py::arg("out"), py::arg("insert") = true,
           py::arg("buf") = 0, py::arg("offsets") = std::vector<int64_t>(),
           py::arg("keep_weights") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("w_forward",
           [](Engine& e, const BatchView& b, uintptr_t pulled, int64_t n_send, uintptr_t pctr,
              int wb) { e.w_forward(b, P<const float>(pulled), n_send, P<float>(pctr), wb); },
           py::arg("batch"), py::arg("pulled"), py::arg("n_send"), py::arg("pctr"),
           py::arg("wb") = 0, py::call_guard<py::gil_scoped_release>())
      .def("w_forward_backward",
           [](Engine& e, const BatchView& b, uintptr_t pulled, int64_t n_send, uintptr_t grads,
              uintptr_t masks, int S, int wb, int group) {
             e.w_forward_backward(b, P<const float>(pulled), n_send, P<float>(grads),
                                  P<u32>(masks), S, wb, group);
           },
           py::arg("batch"), py::arg("pulled"), py::arg("n_send"), py::arg("grads"),
           py::arg("masks"), py::arg("S") = 0, py::arg("wb") = 0, py::arg("group") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("s_apply",
           [](Engine& e, uintptr_t keys, uintptr_t grads, uintptr_t masks,
              std::vector<int64_t> offsets, int S, int buf) {
             e.s_apply(P<const u64>(keys), P<const float>(grads), P<const u32>(masks), offsets, S,
                       buf);
           },
           py::arg("keys"), py::arg("grads"), py::arg("masks"), py::arg("offsets"), py::arg("S"),
           py::arg("buf") = 0, py::call_guard<py::gil_scoped_release>())
      .def("w_forward_backward_csr",
           [](Engine& e, const BatchView& b, uintptr_t pulled, int64_t n_send, int S, int wb,
              uintptr_t cnt, uintptr_t ent, uintptr_t counts, int world, uintptr_t totals) {
             e.w_forward_backward_csr(b, P<const float>(pulled), n_send, S, wb, true, P<u32>(cnt),
                                      P<void>(ent), P<const int64_t>(counts), world, false,
                                      P<int64_t>(totals));
           },
           py::arg("batch"), py::arg("pulled"), py::arg("n_send"), py::arg("S"), py::arg("wb"),
           py::arg("cnt"), py::arg("ent"), py::arg("counts"), py::arg("world"), py::arg("totals"),
           py::call_guard<py::gil_scoped_release>())
      .def("s_apply_csr",
           [](Engine& e, uintptr_t keys, uintptr_t cnt, uintptr_t ent, std::vector<int64_t> offsets,
              int S, int buf) {
             e.s_apply_csr(P<const u64>(keys), P<const u32>(cnt), P<const void>(ent), offsets, S, buf);
           },
           py::arg("keys"), py::arg("cnt"), py::arg("ent"), py::arg("offsets"), py::arg("S"),
           py::arg("buf") = 0, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("csr_entry_bytes", &Engine::csr_entry_bytes)
      .def("csr_exchange", [](Engine& e, int S) {
        return e.csr_slog2(S) >= 0 && e.backend().csr_exchange();
      })
      .def("w_finish", &Engine::w_finish, py::call_guard<py::gil_scoped_release>())
      .def("unpack_block",
           [](Engine& e, uintptr_t block, int64_t rows, std::vector<int> width,
              std::vector<int64_t> col_off, std::vector<uintptr_t> dict, std::vector<int> fgid_col,
              uintptr_t keys, uintptr_t labels, uintptr_t fgid) {
             const size_t F = width.size();
             if (F == 0 || F > (size_t)kMaxPackedFields || col_off.size() != F || dict.size() != F ||
                 fgid_col.size() != F)
               throw std::invalid_argument("unpack_block: one width / offset / dict / fgid per field");
             UnpackArgs a;
             a.block = P<const uint8_t>(block);
             a.rows = rows;
             a.F = (int)F;
             for (size_t f = 0; f < F; ++f) {
               a.width[f] = width[f];
               a.col_off[f] = col_off[f];
               a.dict[f] = P<const u64>(dict[f]);
               a.fgid_col[f] = fgid_col[f];
             }
             a.keys = P<u64>(keys);
             a.labels = P<float>(labels);
             a.fgid = P<int32_t>(fgid);
             e.backend().unpack_block(a);
           },
           py::arg("block"), py::arg("rows"), py::arg("width"), py::arg("col_off"),
           py::arg("dict"), py::arg("fgid_col"), py::arg("keys"), py::arg("labels"),
           py::arg("fgid") = 0, py::call_guard<py::gil_scoped_release>())
      .def("field_major",
           [](Engine& e, uintptr_t src, uintptr_t dst, int64_t rows, int F, int elem_bytes,
              bool widen) {
             e.backend().field_major(P<const void>(src), P<void>(dst), rows, F, elem_bytes, widen);
           },
           py::arg("src"), py::arg("dst"), py::arg("rows"), py::arg("F"), py::arg("elem_bytes"),
           py::arg("widen") = false, py::call_guard<py::gil_scoped_release>())
      .def("read_stats",
           [](Engine& e, bool reset, int which) { return stats_dict(e.read_stats(reset, which)); },
           py::arg("reset") = false, py::arg("which") = 0)
      .def("csr_debug",
           [](Engine& e) {
             std::vector<u32> o, c, w;
             e.csr_debug(o, c, w);
             return py::make_tuple(to_np(o), to_np(c), to_np(w));
           })
      .def("n_unique", &Engine::n_unique)
      .def("table_size", &Engine::table_size)
      .def("scratch_capacity", &Engine::scratch_capacity)
      .def("overflowed", &Engine::overflowed)
      .def("nonzero_weights", &Engine::nonzero_weights)
      .def("export_table",
           [](Engine& e) {
             // straight into the returned arrays (no zero-fill, no extra copy)
             const int64_t n = e.table_size();
             py::array_t<uint64_t> k((py::ssize_t)n);
             py::array_t<uint32_t> w((py::ssize_t)(n * e.state_words()));
             u64* kp = reinterpret_cast<u64*>(k.mutable_data());
             u32* wp = reinterpret_cast<u32*>(w.mutable_data());
             {
               py::gil_scoped_release nogil;
               e.export_into(kp, wp, n);
             }
             return py::make_tuple(k, w);
           })
      .def("import_table",
           [](Engine& e, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> keys,
              py::array_t<uint32_t, py::array::c_style | py::array::forcecast> words) {
             const int64_t n = (int64_t)keys.size();
             if ((int64_t)words.size() != n * e.state_words())
               throw std::invalid_argument("import_table: size mismatch");
             const u64* kp = reinterpret_cast<const u64*>(keys.data());
             const u32* wp = reinterpret_cast<const u32*>(words.data());
             py::gil_scoped_release nogil;
             e.import_from(kp, wp, n);
           })
      .def("save", &Engine::save, py::call_guard<py::gil_scoped_release>())
      .def("load", &Engine::load, py::call_guard<py::gil_scoped_release>())
      .def("synth_batch",
           [](Engine& e, int64_t rows, std::vector<uint64_t> vocab, std::vector<float> zipf,
              uint64_t hash_space, uint64_t seed, uint64_t step, float scale, float bias,
              int64_t slice_rows, uintptr_t keys, uintptr_t labels, uintptr_t fgid,
              bool field_major) {
             SynthArgs a;
             a.col_stride = field_major ? rows : 0;
             a.keys = P<u64>(keys);
             a.labels = P<float>(labels);
             a.fgid = P<int32_t>(fgid);
             a.rows = rows;
             a.fields = (int)vocab.size();
             a.vocab = vocab.data();
             a.zipf_s = zipf.data();
             a.hash_space = hash_space;
             a.seed = seed;
             a.step = step;
             a.planted_scale = scale;
             a.planted_bias = bias;
             return e.synth_batch(a, slice_rows);
           },
           py::arg("rows"), py::arg("vocab"), py::arg("zipf"), py::arg("hash_space"),
           py::arg("seed"), py::arg("step"), py::arg("scale"), py::arg("bias"),
           py::arg("slice_rows"), py::arg("keys") = 0, py::arg("labels") = 0,
           py::arg("fgid") = 0, py::arg("field_major") = false)
      .def("stage_host_batch",
           [](Engine& e, py::array_t<uint64_t> keys, py::object row_ptr, py::object fgid,
              py::array_t<float> labels, int nnz_per_row, int64_t slice_rows) {
             BatchView h;
             h.keys = keys.data();
             h.nnz = keys.size();
             h.labels = labels.data();
             h.rows = labels.size();
             std::vector<int32_t> rp, fg;
             if (!row_ptr.is_none()) {
               auto a = row_ptr.cast<py::array_t<int32_t>>();
               rp.assign(a.data(), a.data() + a.size());
               h.row_ptr = rp.data();
             }
             if (!fgid.is_none()) {
               auto a = fgid.cast<py::array_t<int32_t>>();
               fg.assign(a.data(), a.data() + a.size());
               h.fgid = fg.data();
             }
             h.nnz_per_row = nnz_per_row;
             h.slice_rows = slice_rows;
             return e.stage_host_batch(h);
           });

  py::class_<BlockReader>(m, "BlockReader")
      .def(py::init<const std::string&, size_t>())
      .def("next",
           [](BlockReader& r) -> py::object {
             CsrBlock b;
             if (!r.next(b)) return py::none();
             return block_to_dict(b);
           })
      .def("rewind", &BlockReader::rewind)
      .def_property("parse_threads", &BlockReader::parse_threads, &BlockReader::set_parse_threads);

  py::class_<PrefetchReader>(m, "PrefetchReader")
      .def(py::init<const std::string&, size_t>())
      .def("next", [](PrefetchReader& r) -> py::object {
        CsrBlock b;
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = r.next(b);
        }
        if (!ok) return py::none();
        return block_to_dict(b);
      });

  py::class_<LoadData>(m, "LoadData")
      .def(py::init([](const std::string& p, size_t bs) { return new LoadData(p.c_str(), bs); }))
      .def("load_minibatch_hash_data_fread", &LoadData::load_minibatch_hash_data_fread)
      .def("load_all_data", &LoadData::load_all_data)
      .def("load_minibatch_data", &LoadData::load_minibatch_data)
      .def("load_all_hash_data", &LoadData::load_all_hash_data)
      .def("load_mibibatch_hash_data", &LoadData::load_mibibatch_hash_data)
      .def_property_readonly("label", [](LoadData& l) { return l.m_data.label; })
      .def_property_readonly("fea_matrix", [](LoadData& l) {
        py::list rows;
        for (auto& r : l.m_data.fea_matrix) {
          py::list row;
          for (auto& f : r) row.append(py::make_tuple(f.fgid, (uint64_t)f.fid));
          rows.append(row);
        }
        return rows;
      });

  py::class_<Trainer>(m, "Trainer")
      .def(py::init([](py::dict d) {
        TrainerConfig c;
        c.train_prefix = d["train_prefix"].cast<std::string>();
        c.test_prefix = d["test_prefix"].cast<std::string>();
        if (d.contains("model")) c.model = d["model"].cast<int>();
        if (d.contains("epochs")) c.epochs = d["epochs"].cast<int>();
        if (d.contains("threads")) c.threads = d["threads"].cast<int>();
        if (d.contains("train_block_bytes")) c.train_block_bytes = d["train_block_bytes"].cast<int64_t>();
        if (d.contains("test_block_bytes")) c.test_block_bytes = d["test_block_bytes"].cast<int64_t>();
        if (d.contains("serial_slices")) c.serial_slices = d["serial_slices"].cast<bool>();
        if (d.contains("keep_remainder")) c.keep_remainder = d["keep_remainder"].cast<bool>();
        if (d.contains("mvm_predict_compat")) c.mvm_predict_compat = d["mvm_predict_compat"].cast<bool>();
        if (d.contains("init_push")) c.init_push = d["init_push"].cast<bool>();
        if (d.contains("rank")) c.rank = d["rank"].cast<int>();
        if (d.contains("pred_dir")) c.pred_dir = d["pred_dir"].cast<std::string>();
        if (d.contains("device")) c.device = d["device"].cast<int>();
        if (d.contains("table_log2_cap")) c.table_log2_cap = d["table_log2_cap"].cast<int>();
        if (d.contains("sum_slices")) c.sum_slices = d["sum_slices"].cast<bool>();
        if (d.contains("verbose")) c.verbose = d["verbose"].cast<bool>();
        if (d.contains("model_spec")) c.model_spec = model_from(d["model_spec"].cast<py::dict>());
        if (d.contains("opt")) c.opt = opt_from(d["opt"].cast<py::dict>());
        return new Trainer(c);
      }))
      .def("train", &Trainer::train, py::call_guard<py::gil_scoped_release>())
      .def("train_epochs", &Trainer::train_epochs, py::call_guard<py::gil_scoped_release>())
      .def("predict",
           [](Trainer& t, int block) {
             EvalResult r;
             {
               py::gil_scoped_release rel;
               r = t.predict(block);
             }
             py::dict d;
             d["logloss_printed"] = r.logloss_printed;
             d["ln_logloss"] = r.ln_logloss;
             d["auc"] = r.auc;
             d["tp"] = r.tp;
             d["n"] = r.n;
             d["line"] = r.line;
             return d;
           },
           py::arg("block") = 0)
      .def_property_readonly("threads", &Trainer::threads)
      .def_property_readonly("engine", &Trainer::engine, py::return_value_policy::reference_internal);
}
