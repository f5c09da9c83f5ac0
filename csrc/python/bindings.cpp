// Python bindings (pybind11) for the native mcg runtime:
//   - problem specs, partition / halo plans, host CSR (CPU tests)
//   - CPU reference CG (single process and P virtual ranks)
//   - RCCL communicator + distributed GPU solver
//   - raw-pointer kernel entry points used by cuda_mpi_parallel_amd.ops (the
//     Python side passes torch tensors' data_ptr() and the current HIP stream)
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <chrono>
#include <cstring>
#include <pybind11/stl.h>
#include <thread>

#include <memory>

#include "mcg/cg.hpp"
#include "mcg/check.hpp"
#include "mcg/comm.hpp"
#include "mcg/kernels.hpp"
#include "mcg/local_ranks.hpp"
#include "mcg/matrix.hpp"
#include "mcg/partition.hpp"
#include "mcg/solver.hpp"

namespace py = pybind11;
using namespace mcg;

namespace {

ProblemSpec make_spec(const std::string& problem, int64_t n, int64_t rows, int64_t band, double density,
                      uint64_t seed, const std::string& rhs, int64_t spread, int scramble, int coef) {
  ProblemSpec s;
  s.kind = parse_problem_kind(problem);
  s.N = n;
  s.rows = rows;
  s.band = band;
  s.density = density;
  s.seed = seed;
  s.rhs = parse_rhs_kind(rhs);
  s.spread = spread;
  s.scramble = scramble;
  MCG_CHECK(scramble == 0 || s.kind == ProblemKind::RandomSPD, "scramble: random-SPD family only");
  s.coef = coef;
  MCG_CHECK(coef == 0 || ((coef == 1) && (s.kind == ProblemKind::Poisson2D || s.kind == ProblemKind::Poisson3D)),
            "coef: 0 (constant) or 1 (random conductivity field), Poisson families only");
  if (s.kind == ProblemKind::Demo) s.N = 3;
  return s;
}

CgOptions make_opts(int maxit, double tol, int check_every, bool overlap, bool use_graph, bool force_comm,
                    const std::string& format, int blocks_per_cu, int spmv_variant, int recurrence) {
  CgOptions o;
  o.maxit = maxit;
  o.tol = tol;
  o.check_every = check_every;
  o.overlap = overlap;
  o.use_graph = use_graph;
  o.force_comm = force_comm;
  if (format == "csr") o.format = 0;
  else if (format == "sell" || format == "sell64") o.format = 1;
  else if (format == "sell16" || format == "sell64-d16") o.format = 2;
  else if (format == "sellc8" || format == "sell64-c8") o.format = 3;
  else fail("unknown format: " + format);
  o.blocks_per_cu = blocks_per_cu;
  o.spmv_variant = spmv_variant;
  o.recurrence = recurrence;
  return o;
}

py::dict result_dict(const CgResult& r) {
  py::dict d;
  d["iterations"] = r.iterations;
  d["converged"] = r.converged;
  d["breakdown"] = r.breakdown;
  d["rnorm"] = r.rnorm;
  d["beta_clamps"] = r.beta_clamps;
  d["rr0_local"] = r.rr0_local;
  d["setup_seconds"] = r.setup_seconds;
  d["solve_seconds"] = r.solve_seconds;
  d["iters_per_second"] = r.iters_per_second();
  return d;
}

py::dict layout_dict(const LocalLayout& L) {
  py::dict d;
  d["rank"] = L.rank;
  d["world"] = L.world;
  d["n_global"] = L.n_global;
  d["row_begin"] = L.row_begin;
  d["row_end"] = L.row_end;
  d["col_lo"] = L.col_lo;
  d["col_hi"] = L.col_hi;
  d["pad"] = L.pad;
  d["ext_len"] = L.ext_len;
  d["own_off"] = L.own_off;
  d["interior_begin"] = L.interior_begin;
  d["interior_end"] = L.interior_end;
  d["allgather"] = L.allgather;
  d["block"] = L.block;
  py::list sends, recvs;
  for (auto& h : L.sends) sends.append(py::make_tuple(h.peer, h.gbegin, h.count));
  for (auto& h : L.recvs) recvs.append(py::make_tuple(h.peer, h.gbegin, h.count));
  d["sends"] = sends;
  d["recvs"] = recvs;
  return d;
}

template <typename T>
py::array_t<T> to_numpy(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<std::vector<T>*>(p); });
  return py::array_t<T>(heap->size(), heap->data(), owner);
}

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "mcg: MI355X-native distributed conjugate-gradient runtime (HIP + RCCL)";

  static py::exception<Error> mcg_error(m, "MCGError");
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const Error& e) {
      const std::string msg = e.detail().empty() ? std::string(e.what()) : std::string(e.what()) + " [" + e.detail() + "]";
      py::set_error(mcg_error, msg.c_str());
    }
  });

  py::class_<ProblemSpec>(m, "ProblemSpec")
      .def(py::init(&make_spec), py::arg("problem") = "demo", py::arg("n") = 3, py::arg("rows") = 0,
           py::arg("band") = 0, py::arg("density") = 0.5, py::arg("seed") = 1234, py::arg("rhs") = "reference",
           py::arg("spread") = 0, py::arg("scramble") = 0, py::arg("coef") = 0)
      .def_property_readonly("name", [](const ProblemSpec& s) { return problem_name(s); })
      .def_property_readonly("n_rows", [](const ProblemSpec& s) { return global_rows(s); })
      .def_property_readonly("bandwidth", [](const ProblemSpec& s) { return bandwidth(s); })
      .def_property_readonly("closed_form_nnz", [](const ProblemSpec& s) { return closed_form_nnz(s); })
      .def_readonly("N", &ProblemSpec::N)
      .def_readonly("rows", &ProblemSpec::rows)
      .def_readonly("band", &ProblemSpec::band)
      .def_readonly("density", &ProblemSpec::density)
      .def_readonly("seed", &ProblemSpec::seed)
      .def_readonly("spread", &ProblemSpec::spread)
      .def_readonly("scramble", &ProblemSpec::scramble)
      .def_readonly("coef", &ProblemSpec::coef)
      .def("perm", [](const ProblemSpec& s, int64_t i, bool inverse) {
        MCG_CHECK(scrambled(s) && i >= 0 && i < s.rows, "perm: scrambled random SPD, 0 <= i < rows");
        return inverse ? scramble_inv(s, i) : scramble_fwd(s, i);
      }, py::arg("i"), py::arg("inverse") = false, "pi(i) (base row of scrambled row i) or pi^-1(i)")
      .def("row_length", [](const ProblemSpec& s, int64_t i) { return row_length(s, i); })
      .def("rhs_value", [](const ProblemSpec& s, int64_t i) { return rhs_value(s, i); })
      .def("row", [](const ProblemSpec& s, int64_t i) {
        py::list cols, vals;
        for_each_entry(s, i, [&](int64_t c, double v) { cols.append(c); vals.append(v); });
        return py::make_tuple(cols, vals);
      });

  // ---- user matrices (kind csr) ----
  py::class_<HostMatrix, std::shared_ptr<HostMatrix>>(m, "HostMatrix")
      .def(py::init([](py::array_t<int64_t, py::array::c_style | py::array::forcecast> indptr,
                       py::array_t<int64_t, py::array::c_style | py::array::forcecast> indices,
                       py::array_t<double, py::array::c_style | py::array::forcecast> data, py::object b) {
             std::vector<int64_t> rp(indptr.data(), indptr.data() + indptr.size());
             std::vector<int64_t> ci(indices.data(), indices.data() + indices.size());
             std::vector<double> v(data.data(), data.data() + data.size());
             std::vector<double> bv;
             if (!b.is_none()) {
               auto ba = py::array_t<double, py::array::c_style | py::array::forcecast>::ensure(b);
               if (!ba) throw py::value_error("b must be a float64 vector");
               bv.assign(ba.data(), ba.data() + ba.size());
             }
             const int64_t n = (int64_t)rp.size() - 1;
             py::gil_scoped_release rel;
             return std::make_shared<HostMatrix>(n, std::move(rp), std::move(ci), std::move(v), std::move(bv));
           }),
           py::arg("indptr"), py::arg("indices"), py::arg("data"), py::arg("b") = py::none(),
           "0-based CSR (int64 row pointers / columns, float64 values), optional right-hand side b")
      .def_static("read_mtx", [](const std::string& path) {
        py::gil_scoped_release rel;
        return std::shared_ptr<HostMatrix>(read_matrix_market(path));
      }, "Matrix Market coordinate file (general / symmetric / skew-symmetric; real / integer / pattern)")
      .def_property_readonly("n", &HostMatrix::n)
      .def_property_readonly("nnz", &HostMatrix::nnz)
      .def_property_readonly("bandwidth", [](const HostMatrix& a) { return a.view().bw; })
      .def_property_readonly("far_entries", [](const HostMatrix& a) { return a.view().far; })
      .def_property_readonly("stencil_line", [](const HostMatrix& a) { return a.view().line; })
      .def_property_readonly("stencil_plane", [](const HostMatrix& a) { return a.view().plane; })
      .def_property_readonly("has_rhs", [](const HostMatrix& a) { return !a.rhs().empty(); })
      .def("symmetric", &HostMatrix::symmetric_pattern_and_values)
      .def("spec", [](const HostMatrix& a, const std::string& rhs, uint64_t seed) {
        return a.spec(parse_rhs_kind(rhs), seed);
      }, py::arg("rhs") = "reference", py::arg("seed") = 1234, py::keep_alive<0, 1>(),
         "ProblemSpec of kind csr over this matrix (the spec keeps the matrix alive)");
  m.def("read_vector", &read_vector, "dense vector: Matrix Market array file or one value per line");

  // the pass-form overrides and test hooks live in CgOptions::form / ::hooks (cg.hpp); Python sees
  // them as flat attributes of CgOptions (opts.carry = 0), the C++ CLI as --carry / --pmat / ...
#define MCG_FORM_PROP(n) \
  .def_property(#n, [](const CgOptions& o) { return o.form.n; }, [](CgOptions& o, decltype(PassForm::n) v) { o.form.n = v; })
#define MCG_HOOK_PROP(n) \
  .def_property(#n, [](const CgOptions& o) { return o.hooks.n; }, [](CgOptions& o, decltype(TestHooks::n) v) { o.hooks.n = v; })
  py::class_<CgOptions>(m, "CgOptions")
      .def(py::init(&make_opts), py::arg("maxit") = 2000, py::arg("tol") = 1e-7, py::arg("check_every") = 32,
           py::arg("overlap") = true, py::arg("use_graph") = true, py::arg("force_comm") = false,
           py::arg("format") = "csr", py::arg("blocks_per_cu") = 0, py::arg("spmv_variant") = -1,
           py::arg("recurrence") = 0)
      .def_readwrite("recurrence", &CgOptions::recurrence)
      MCG_FORM_PROP(interleave)
      MCG_FORM_PROP(window)
      MCG_FORM_PROP(pipeline)
      MCG_FORM_PROP(carry)
      MCG_FORM_PROP(fused_reduce)
      MCG_FORM_PROP(tiles)
      MCG_FORM_PROP(tile_seg_log2)
      MCG_FORM_PROP(tile_waves)
      MCG_FORM_PROP(carry_vc)
      MCG_FORM_PROP(lean_split)
      MCG_FORM_PROP(halo_pull)
      MCG_FORM_PROP(p3buf)
      .def_readwrite("pipe_rr", &CgOptions::pipe_rr)
      .def_readwrite("graph_iters", &CgOptions::graph_iters)
      .def_readwrite("placement_tries", &CgOptions::placement_tries)
      .def_readwrite("placement_leads", &CgOptions::placement_leads)
      .def_readwrite("halo_mode", &CgOptions::halo_mode)
      MCG_FORM_PROP(pmat)
      MCG_FORM_PROP(sell_sigma)
      MCG_FORM_PROP(sell_aligned)
      MCG_FORM_PROP(ag_overlap)
      MCG_FORM_PROP(halo_ahead)
      MCG_FORM_PROP(ap_recompute)
      MCG_FORM_PROP(carry_dia)
      MCG_FORM_PROP(p3)
      MCG_FORM_PROP(dia_uniform)
      MCG_HOOK_PROP(fail_graph_launch_at)
      .def_readwrite("checkpoint_every", &CgOptions::checkpoint_every)
      .def_readwrite("checkpoint_path", &CgOptions::checkpoint_path)
      MCG_HOOK_PROP(force_idx64)
      MCG_HOOK_PROP(inject_nan_at)
      MCG_HOOK_PROP(lean_packed)
      MCG_HOOK_PROP(gen_piece_lines)
      MCG_HOOK_PROP(split_serial)
      MCG_HOOK_PROP(pull_proxy)
      MCG_HOOK_PROP(probe_pick_halo)
      MCG_HOOK_PROP(probe_pick_ar)
      .def_readwrite("transport_probe", &CgOptions::transport_probe)
      .def_readwrite("spmv_variant", &CgOptions::spmv_variant)
      .def_readwrite("maxit", &CgOptions::maxit)
      .def_readwrite("tol", &CgOptions::tol)
      .def_readwrite("rtol", &CgOptions::rtol)
      .def_readwrite("watchdog_seconds", &CgOptions::watchdog_seconds)
      .def_readwrite("check_every", &CgOptions::check_every)
      .def_readwrite("reserve_cus", &CgOptions::reserve_cus)
      .def_readwrite("overlap", &CgOptions::overlap)
      .def_readwrite("use_graph", &CgOptions::use_graph)
      .def_readwrite("force_comm", &CgOptions::force_comm)
      .def_readwrite("format", &CgOptions::format)
      .def_readwrite("blocks_per_cu", &CgOptions::blocks_per_cu);
#undef MCG_FORM_PROP
#undef MCG_HOOK_PROP

  // ---- partition / halo plan / host CSR ----
  m.def("partition_rows", [](const ProblemSpec& s, int world, int halo_mode) {
    return partition_rows(s, world, halo_mode).offsets;
  }, py::arg("spec"), py::arg("world"), py::arg("halo_mode") = -1);
  m.def("partition_by_weight", [](const std::vector<int64_t>& prefix, int world) {
    return partition_by_weight(prefix, world).offsets;
  });
  m.def("make_layout", [](const ProblemSpec& s, int world, int rank, int halo_mode) {
    return layout_dict(make_layout(s, partition_rows(s, world, halo_mode), rank));
  }, py::arg("spec"), py::arg("world"), py::arg("rank"), py::arg("halo_mode") = -1);
  m.def("host_csr", [](const ProblemSpec& s, int world, int rank) {
    LocalLayout L = make_layout(s, partition_rows(s, world), rank);
    HostCsr A = build_local_csr(s, L);
    return py::make_tuple(to_numpy(std::move(A.rowptr)), to_numpy(std::move(A.cols)), to_numpy(std::move(A.vals)));
  }, py::arg("spec"), py::arg("world") = 1, py::arg("rank") = 0);
  m.def("host_rhs", [](const ProblemSpec& s, int64_t r0, int64_t r1) { return to_numpy(build_rhs(s, r0, r1)); });

  // ---- CPU reference path ----
  m.def("cpu_cg", [](const ProblemSpec& s, const CgOptions& o) {
    std::vector<double> x, hist;
    CgResult r;
    {
      py::gil_scoped_release rel;
      r = cpu_cg(s, o, &x, &hist);
    }
    py::dict d = result_dict(r);
    d["x"] = to_numpy(std::move(x));
    d["rnorm_history"] = to_numpy(std::move(hist));
    return d;
  });
  m.def("cpu_cg_partitioned", [](const ProblemSpec& s, int world, const CgOptions& o) {
    std::vector<double> x, hist;
    CgResult r;
    {
      py::gil_scoped_release rel;
      r = cpu_cg_partitioned(s, world, o, &x, &hist);
    }
    py::dict d = result_dict(r);
    d["x"] = to_numpy(std::move(x));
    d["rnorm_history"] = to_numpy(std::move(hist));
    return d;
  });

  // ---- device / RCCL ----
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    (void)hipGetLastError();
    return n;
  });
  m.def("unique_id", []() { return py::bytes(unique_id_bytes()); });
  m.def("rccl_info", []() {
    py::dict d;
    d["version"] = rccl_version();
    d["library"] = rccl_library();
    return d;
  }, "ncclGetVersion and the library that provides it (the same RCCL as bin/mcg-cg: tests/test_gpu_rccl.py)");

  py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
      .def(py::init([](int rank, int world, py::bytes id_red, py::bytes id_halo) {
             std::string a = id_red, b = id_halo;
             py::gil_scoped_release rel;
             return std::make_shared<Comm>(rank, world, unique_id_from_bytes(a), unique_id_from_bytes(b));
           }),
           py::arg("rank"), py::arg("world"), py::arg("reduce_id"), py::arg("halo_id"))
      .def(py::init([](int rank, int world, py::bytes id) {
             std::string a = id;
             py::gil_scoped_release rel;
             return std::make_shared<Comm>(rank, world, unique_id_from_bytes(a));
           }),
           py::arg("rank"), py::arg("world"), py::arg("id"),
           "single-communicator mode: halo and all-reduce on one communicator, issued in one stream order")
      .def_property_readonly("serialized", &Comm::serialized)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("world", &Comm::world)
      .def_property_readonly("count", &Comm::count)
      .def("allreduce_sum_ptr", [](Comm& c, uintptr_t buf, size_t count, uintptr_t stream) {
        c.allreduce_sum(reinterpret_cast<double*>(buf), count, as_stream(stream));
      })
      .def("sendrecv_ptr", [](Comm& c, uintptr_t send, int to, uintptr_t recv, int from, size_t n, uintptr_t stream) {
        c.sendrecv(reinterpret_cast<const double*>(send), to, reinterpret_cast<double*>(recv), from, n,
                   as_stream(stream));
      })
      .def("allgather_inplace_ptr", [](Comm& c, uintptr_t buf, size_t block, uintptr_t stream) {
        c.allgather_inplace(reinterpret_cast<double*>(buf), block, as_stream(stream));
      })
      .def("check_async", &Comm::check_async)
      .def("abort", &Comm::abort);

  py::class_<NullComm, std::shared_ptr<NullComm>>(m, "NullComm",
                                                  "one rank of a P-rank run with collectives that move nothing "
                                                  "(per-rank timing rehearsal on one GPU)")
      .def(py::init<int, int>(), py::arg("rank"), py::arg("world"));

  py::class_<DelayComm, std::shared_ptr<DelayComm>>(m, "DelayComm",
                                                    "one rank of a P-rank run whose all-reduce / halo cost a fixed "
                                                    "device-side delay and move nothing (latency rehearsal)")
      .def(py::init<int, int, double, double, bool, bool>(), py::arg("rank"), py::arg("world"), py::arg("allreduce_us"),
           py::arg("halo_us") = 0.0, py::arg("fat") = false, py::arg("copy_halo") = false,
           "copy_halo: the halo as copy-engine (NoCU) copies of the layout's message sizes instead of a spin");

  py::class_<PeerHaloComm, std::shared_ptr<PeerHaloComm>>(
      m, "PeerHaloComm",
      "the halo on copy engines (IPC-mapped peer buffers, flags by stream memory operations); the all-reduce "
      "goes to the wrapped communicator")
      .def(py::init([](std::shared_ptr<Comm> c, int rank, int world) { return std::make_shared<PeerHaloComm>(c, rank, world); }),
           py::arg("inner"), py::arg("rank"), py::arg("world"))
      .def(py::init([](std::shared_ptr<NullComm> c, int rank, int world) { return std::make_shared<PeerHaloComm>(c, rank, world); }),
           py::arg("inner"), py::arg("rank"), py::arg("world"))
      .def(py::init([](std::shared_ptr<DelayComm> c, int rank, int world) { return std::make_shared<PeerHaloComm>(c, rank, world); }),
           py::arg("inner"), py::arg("rank"), py::arg("world"))
      .def("local_handles", [](const PeerHaloComm& c) { return py::bytes(c.local_handles()); })
      .def("attach", [](PeerHaloComm& c, const std::vector<py::bytes>& all) {
        std::vector<std::string> v;
        for (const py::bytes& b : all) v.push_back(std::string(b));
        c.attach(v);
      })
      .def_property_readonly("attached", &PeerHaloComm::attached)
      .def("mailbox_handle", [](PeerHaloComm& c) { return py::bytes(c.mailbox_handle()); })
      .def("attach_mailbox", [](PeerHaloComm& c, const std::vector<py::bytes>& all) {
        std::vector<std::string> v;
        for (const py::bytes& b : all) v.push_back(std::string(b));
        c.attach_mailbox(v);
      }, "map every rank's IPC all-reduce mailbox; from then on the all-reduce runs through them")
      .def_property("ipc_allreduce", &PeerHaloComm::ipc_allreduce, &PeerHaloComm::use_alt_allreduce,
                    "the all-reduce runs through the mapped mailboxes (settable once attach_mailbox ran; the "
                    "solver's transport probe may change it at the first reset)")
      .def_property("halo_via_inner", &PeerHaloComm::halo_via_inner, &PeerHaloComm::set_halo_via_inner)
      .def_readwrite("ar_budget_seconds", &PeerHaloComm::ar_budget_seconds)
      .def("allreduce_ptr", [](PeerHaloComm& c, uintptr_t buf, size_t count, uintptr_t stream) {
        c.allreduce_sum(reinterpret_cast<double*>(buf), count, as_stream(stream));
      }, "test hook: in-place sum all-reduce of `count` doubles at a device pointer")
      .def("check_async", &PeerHaloComm::check_async)
      .def("set_capturable", &PeerHaloComm::set_capturable)
      .def("peer_buffers", &PeerHaloComm::peer_buffers)
      .def("register_halo_buffers", [](PeerHaloComm& c, const std::vector<uintptr_t>& bufs, int64_t own_off, int64_t row_begin) {
        std::vector<double*> v;
        for (uintptr_t b : bufs) v.push_back(reinterpret_cast<double*>(b));
        c.register_halo_buffers(v, own_off, row_begin);
      })
      .def("halo_exchange_ptrs", [](PeerHaloComm& c, const ProblemSpec& s, const std::vector<uintptr_t>& vecs,
                                    uintptr_t stream) {
        const LocalLayout L = make_layout(s, partition_rows(s, c.world()), c.rank());
        std::vector<double*> v;
        for (uintptr_t b : vecs) v.push_back(reinterpret_cast<double*>(b));
        c.halo_exchange(L, v.data(), (int)v.size(), as_stream(stream));
      }, "test hook: one halo exchange of ext-layout vectors laid out for (spec, world, rank)");

  py::class_<GpuCgSolver>(m, "Solver")
      .def(py::init([](const ProblemSpec& s, const CgOptions& o, int rank, int world, std::shared_ptr<Comm> comm) {
             return new GpuCgSolver(s, o, rank, world, comm.get());
           }),
           py::arg("spec"), py::arg("opts"), py::arg("rank") = 0, py::arg("world") = 1,
           py::arg("comm") = nullptr, py::keep_alive<1, 6>(), py::keep_alive<1, 2>())
      .def(py::init([](const ProblemSpec& s, const CgOptions& o, int rank, int world, std::shared_ptr<NullComm> comm) {
             return new GpuCgSolver(s, o, rank, world, comm.get());
           }),
           py::arg("spec"), py::arg("opts"), py::arg("rank"), py::arg("world"), py::arg("comm"),
           py::keep_alive<1, 6>(), py::keep_alive<1, 2>())
      .def(py::init([](const ProblemSpec& s, const CgOptions& o, int rank, int world, std::shared_ptr<DelayComm> comm) {
             return new GpuCgSolver(s, o, rank, world, comm.get());
           }),
           py::arg("spec"), py::arg("opts"), py::arg("rank"), py::arg("world"), py::arg("comm"),
           py::keep_alive<1, 6>(), py::keep_alive<1, 2>())
      .def(py::init([](const ProblemSpec& s, const CgOptions& o, int rank, int world, std::shared_ptr<PeerHaloComm> comm) {
             return new GpuCgSolver(s, o, rank, world, comm.get());
           }),
           py::arg("spec"), py::arg("opts"), py::arg("rank"), py::arg("world"), py::arg("comm"),
           py::keep_alive<1, 6>(), py::keep_alive<1, 2>())
      .def("setup", [](GpuCgSolver& g) { py::gil_scoped_release rel; g.setup(); })
      .def("reset", [](GpuCgSolver& g) { py::gil_scoped_release rel; g.reset(); })
      .def("solve", [](GpuCgSolver& g, bool resume) {
        CgResult r;
        {
          py::gil_scoped_release rel;
          r = g.solve(resume);
        }
        return result_dict(r);
      }, py::arg("resume") = false)
      .def("save_checkpoint", [](GpuCgSolver& g, const std::string& p) { py::gil_scoped_release rel; g.save_checkpoint(p); })
      .def("load_checkpoint", [](GpuCgSolver& g, const std::string& p) { py::gil_scoped_release rel; g.load_checkpoint(p); })
      .def("run_iterations", [](GpuCgSolver& g, int k) { py::gil_scoped_release rel; g.run_iterations(k); })
      .def("finalize", &GpuCgSolver::finalize)
      .def("synchronize", [](GpuCgSolver& g) { py::gil_scoped_release rel; g.synchronize(); })
      .def("result", [](GpuCgSolver& g) { return result_dict(g.result()); })
      .def("x_local", [](GpuCgSolver& g) { return to_numpy(g.x_local()); })
      .def("true_residual_norm", [](GpuCgSolver& g) { py::gil_scoped_release rel; return g.true_residual_norm(); })
      .def("phase_profile", [](GpuCgSolver& g, int iters) {
        std::vector<std::pair<std::string, double>> r;
        {
          py::gil_scoped_release rel;
          r = g.phase_profile(iters);
        }
        py::dict d;
        for (auto& kv : r) d[py::str(kv.first)] = kv.second;
        return d;
      })
      .def_property_readonly("iterations_enqueued", &GpuCgSolver::iterations_enqueued)
      .def_property_readonly("stream", [](GpuCgSolver& g) { return reinterpret_cast<uintptr_t>(g.stream()); })
      .def_property_readonly("layout", [](GpuCgSolver& g) { return layout_dict(g.layout()); })
      .def_property_readonly("info", [](GpuCgSolver& g) {
        const SolverInfo& i = g.info();
        py::dict d;
        d["n_global"] = i.n_global;
        d["n_local"] = i.n_local;
        d["nnz_local"] = i.nnz_local;
        d["ext_len"] = i.ext_len;
        d["halo_in"] = i.halo_in;
        d["halo_out"] = i.halo_out;
        d["interior_rows"] = i.interior_rows;
        d["idx64"] = i.idx64;
        d["format"] = i.format == 5 ? "tiles" : i.format == 4 ? "sell64-aligned"
                      : i.format == 3 ? "sell64-c8" : (i.format == 2 ? "sell64-d16" : (i.format == 1 ? "sell64" : "csr"));
        d["recurrence"] = i.recurrence == 2 ? "pipelined" : i.recurrence == 1 ? "single-reduction" : "two-reduction";
        d["pipe_rr"] = i.pipe_rr;
        d["pipe_ar_first"] = i.pipe_ar_first;
        d["pipe_spmv_us"] = i.pipe_spmv_us;
        d["pipe_allreduce_us"] = i.pipe_allreduce_us;
        d["interleave"] = i.interleave;
        d["window"] = i.window;
        d["pipeline"] = i.pipeline;
        d["carry"] = i.carry;
        d["fused_reduce"] = i.fused_reduce;
        d["pmat"] = i.pmat;
        d["tiles"] = i.tiles;
        d["tiles_tu"] = i.tiles_tu;
        d["tile_segments"] = i.tile_segments;
        d["sigma"] = i.sigma;
        d["sell_fill"] = i.sell_fill;
        d["allgather"] = i.allgather;
        d["ag_overlap"] = i.ag_overlap;
        d["halo_ahead"] = i.halo_ahead;
        d["ap_recompute"] = i.ap_recompute;
        d["ag_local_frac"] = i.ag_local_frac;
        d["graph_fallbacks"] = i.graph_fallbacks;
        d["graphs"] = i.graphs;
        d["xcd_map"] = i.xcd_map;
        d["dia4"] = i.dia4;
        d["diav"] = i.diav;
        d["halo_pull"] = i.halo_pull;
        d["p3buf"] = i.p3buf;
        d["aligned_fill"] = i.aligned_fill;
        d["p3"] = i.p3;
        d["dia_uniform"] = i.dia_uniform;
        d["lean_only"] = i.lean_only;
        d["ar3_kw"] = i.ar3_kw;
        d["ar3_runs"] = i.ar3_runs;
        d["carry_xchg"] = i.carry_xchg;
        d["placement_sets"] = i.placement_sets;
        d["placement_gain"] = i.placement_gain;
        d["placement_best_ms"] = i.placement_best_ms;
        d["placement_worst_ms"] = i.placement_worst_ms;
        d["placement_lead_trial"] = i.placement_lead_trial;
        d["placement_peak_bytes"] = i.placement_peak_bytes;
        d["probe_ran"] = i.probe_ran;
        d["probe_pull_us"] = i.probe_pull_us;
        d["probe_xchg_us"] = i.probe_xchg_us;
        d["probe_alt_us"] = i.probe_alt_us;
        d["probe_iters"] = i.probe_iters;
        d["probe_pull_bitwise"] = i.probe_pull_bitwise;
        d["probe_alt_close"] = i.probe_alt_close;
        d["probe_alt_timeout"] = i.probe_alt_timeout;
        d["alt_allreduce"] = i.alt_allreduce;
        d["device_bytes"] = i.device_bytes;
        d["bytes_per_iter_model"] = i.bytes_per_iter_model;
        d["grid_a"] = i.grid_a;
        d["grid_odd"] = i.grid_odd;
        d["lean_mix"] = i.lean_mix;
        d["lean_split"] = i.lean_split;
        d["grid_b"] = i.grid_b;
        d["max_row_len"] = i.max_row_len;
        d["spmv_variant"] = i.spmv_variant;
        d["spmv_param"] = i.spmv_param;
        return d;
      });

  m.def("run_local_ranks", [](const ProblemSpec& s, const CgOptions& o, int world, int fixed_iters, bool verify,
                              int phase_iters) {
    LocalRunResult lr;
    {
      py::gil_scoped_release rel;
      lr = run_local_ranks(s, o, world, fixed_iters, verify, phase_iters);
    }
    py::list ranks;
    std::vector<double> x;
    for (auto& rr : lr.ranks) {
      py::dict d = result_dict(rr.res);
      d["row_begin"] = rr.row_begin;
      d["true_rnorm"] = rr.true_rnorm;
      d["carry"] = rr.carry;
      d["ap_recompute"] = rr.ap_recompute;
      d["lean_only"] = rr.lean_only;
      d["lean_split"] = rr.lean_split;
      d["p3"] = rr.p3;
      d["p3buf"] = rr.p3buf;
      d["dia_uniform"] = rr.dia_uniform;
      d["halo_pull"] = rr.halo_pull;
      d["ag_overlap"] = rr.ag_overlap;
      d["ag_local_frac"] = rr.ag_local_frac;
      d["probe_ran"] = rr.probe_ran;
      d["probe_pull_bitwise"] = rr.probe_pull_bitwise;
      d["probe_pull_us"] = rr.probe_pull_us;
      d["probe_xchg_us"] = rr.probe_xchg_us;
      py::dict ph;
      for (auto& kv : rr.phases) ph[py::str(kv.first)] = kv.second;
      d["phases"] = ph;
      ranks.append(d);
      x.insert(x.end(), rr.x.begin(), rr.x.end());
    }
    py::dict out;
    out["ranks"] = ranks;
    out["x"] = to_numpy(std::move(x));
    return out;
  }, py::arg("spec"), py::arg("opts"), py::arg("world"), py::arg("fixed_iters") = 0, py::arg("verify") = false,
     py::arg("phase_iters") = 0,
     "P ranks as threads on the current device with the in-process LocalComm (multi-rank test harness)");

  // ---- raw-pointer kernel entry points (ops API) ----
  py::module_ k = m.def_submodule("kernels", "hand-written gfx950 kernels on raw device pointers");
  k.def("spmv_csr", [](uintptr_t rowptr, bool idx64, uintptr_t cols, uintptr_t vals, int64_t n_rows, uintptr_t x,
                       uintptr_t y, uintptr_t stream) {
    if (idx64)
      kern::spmv_csr<int64_t>(CsrDev<int64_t>{reinterpret_cast<const int64_t*>(rowptr),
                                              reinterpret_cast<const int32_t*>(cols),
                                              reinterpret_cast<const double*>(vals), n_rows},
                              reinterpret_cast<const double*>(x), reinterpret_cast<double*>(y), as_stream(stream));
    else
      kern::spmv_csr<int32_t>(CsrDev<int32_t>{reinterpret_cast<const int32_t*>(rowptr),
                                              reinterpret_cast<const int32_t*>(cols),
                                              reinterpret_cast<const double*>(vals), n_rows},
                              reinterpret_cast<const double*>(x), reinterpret_cast<double*>(y), as_stream(stream));
  });
  k.def("spmv_sell", [](uintptr_t slice_ptr, uintptr_t cols, uintptr_t vals, int64_t n_rows, uintptr_t x,
                        uintptr_t y, uintptr_t stream) {
    kern::spmv_sell(SellDev{reinterpret_cast<const int64_t*>(slice_ptr), reinterpret_cast<const int32_t*>(cols),
                            reinterpret_cast<const double*>(vals), n_rows},
                    reinterpret_cast<const double*>(x), reinterpret_cast<double*>(y), as_stream(stream));
  });
  // SELL-64/c8 (dictionary codes) from a SELL-64 matrix with int32 columns (own_off = 0):
  // returns (dict as float64 [nv*nd, 2] = {value, int64 offset bits}, nv, nd) or None if it does not fit
  k.def("sell_dict_build", [](uintptr_t slice_ptr, uintptr_t cols, uintptr_t vals, int64_t n_rows,
                              uintptr_t stream) -> py::object {
    SellDev S{reinterpret_cast<const int64_t*>(slice_ptr), reinterpret_cast<const int32_t*>(cols),
              reinterpret_cast<const double*>(vals), n_rows};
    std::vector<double2> dict;
    int nv = 0, nd = 0;
    bool ok;
    {
      py::gil_scoped_release rel;
      ok = kern::sell_dict_build(S, dict, nv, nd, as_stream(stream));
    }
    if (!ok) return py::none();
    py::array_t<double> d({(py::ssize_t)dict.size(), (py::ssize_t)2});
    std::memcpy(d.mutable_data(), dict.data(), dict.size() * sizeof(double2));
    return py::make_tuple(d, nv, nd);
  });
  k.def("sell_to_c8", [](uintptr_t slice_ptr, uintptr_t cols, uintptr_t vals, int64_t n_rows, uintptr_t dict, int nv,
                         int nd, uintptr_t codes, uintptr_t stream) {
    SellDev S{reinterpret_cast<const int64_t*>(slice_ptr), reinterpret_cast<const int32_t*>(cols),
              reinterpret_cast<const double*>(vals), n_rows};
    kern::sell_to_c8(S, reinterpret_cast<const double2*>(dict), nv, nd, reinterpret_cast<uint8_t*>(codes),
                     as_stream(stream));
  });
  k.def("spmv_sell_c8", [](uintptr_t slice_ptr, uintptr_t codes, uintptr_t dict, int ndict, int64_t n_rows,
                           uintptr_t x, uintptr_t y, uintptr_t stream) {
    SellDev S{reinterpret_cast<const int64_t*>(slice_ptr), nullptr, nullptr, n_rows};
    S.codes = reinterpret_cast<const uint8_t*>(codes);
    S.dict = reinterpret_cast<const double2*>(dict);
    S.ndict = ndict;
    kern::spmv_sell(S, reinterpret_cast<const double*>(x), reinterpret_cast<double*>(y), as_stream(stream));
  });
  k.def("csr_to_sell", [](uintptr_t rowptr64, uintptr_t cols, uintptr_t vals, int64_t n, uintptr_t slice_ptr,
                          uintptr_t scols, uintptr_t svals, uintptr_t stream) {
    kern::csr_to_sell<int64_t>(reinterpret_cast<const int64_t*>(rowptr64), reinterpret_cast<const int32_t*>(cols),
                               reinterpret_cast<const double*>(vals), n, 0,
                               reinterpret_cast<const int64_t*>(slice_ptr), reinterpret_cast<int32_t*>(scols),
                               reinterpret_cast<double*>(svals), as_stream(stream));
  });
  k.def("dot_partials", [](uintptr_t a, uintptr_t b, int64_t n, uintptr_t partials, int grid, uintptr_t stream) {
    kern::dot_partials(reinterpret_cast<const double*>(a), reinterpret_cast<const double*>(b), n,
                       reinterpret_cast<double*>(partials), grid, as_stream(stream));
  });
  k.def("sum_partials", [](uintptr_t partials, int np, uintptr_t out, uintptr_t stream) {
    kern::sum_partials(reinterpret_cast<const double*>(partials), np, reinterpret_cast<double*>(out),
                       as_stream(stream));
  });
  k.def("axpy", [](double a, uintptr_t x, uintptr_t y, int64_t n, uintptr_t stream) {
    kern::axpy(a, reinterpret_cast<const double*>(x), reinterpret_cast<double*>(y), n, as_stream(stream));
  });
  k.def("xpby", [](uintptr_t x, double b, uintptr_t y, int64_t n, uintptr_t stream) {
    kern::xpby(reinterpret_cast<const double*>(x), b, reinterpret_cast<double*>(y), n, as_stream(stream));
  });
  k.def("gen_rowlen", [](const ProblemSpec& s, int64_t row_begin, int64_t n, uintptr_t rowptr, uintptr_t stream) {
    kern::gen_rowlen(s, row_begin, n, reinterpret_cast<int64_t*>(rowptr), as_stream(stream));
  });
  k.def("scan_inclusive_i64", [](uintptr_t a, int64_t n, uintptr_t tmp, uintptr_t stream) {
    kern::scan_inclusive_i64(reinterpret_cast<int64_t*>(a), n, reinterpret_cast<int64_t*>(tmp), as_stream(stream));
  });
  k.def("scan_tmp_elems", &kern::scan_tmp_elems);
  k.def("gen_fill", [](const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t col_lo, int64_t pad,
                       uintptr_t rp64, uintptr_t cols, uintptr_t vals, uintptr_t stream) {
    kern::gen_fill<int64_t>(s, row_begin, n, col_lo, pad, reinterpret_cast<const int64_t*>(rp64), nullptr,
                            reinterpret_cast<int32_t*>(cols), reinterpret_cast<double*>(vals), as_stream(stream));
  });
  k.def("gen_rhs", [](const ProblemSpec& s, int64_t row_begin, int64_t n, uintptr_t b, uintptr_t stream) {
    kern::gen_rhs(s, row_begin, n, reinterpret_cast<double*>(b), as_stream(stream));
  });
  k.def("sell_slice_widths", [](uintptr_t rp64, int64_t n, uintptr_t sp, uintptr_t stream) {
    kern::sell_slice_widths(reinterpret_cast<const int64_t*>(rp64), n, reinterpret_cast<int64_t*>(sp),
                            as_stream(stream));
  });
  k.def("grid_for", &kern::grid_for);
  k.def("spin", [](uintptr_t out, double us, bool fat, int blocks, uintptr_t stream, uintptr_t where) {
    kern::spin(reinterpret_cast<double*>(out), us, fat, blocks, as_stream(stream), reinterpret_cast<int*>(where));
  }, py::arg("out"), py::arg("microseconds"), py::arg("fat"), py::arg("blocks"), py::arg("stream"),
     py::arg("where") = 0,
     "probe: workgroups spinning on the realtime clock (fat: ~270 VGPRs per wave live); where: __smid per block");
  k.def("hog", [](uintptr_t out, double us, int blocks, uintptr_t stream, uintptr_t where) {
    kern::hog(reinterpret_cast<double*>(out), us, blocks, as_stream(stream), reinterpret_cast<int*>(where));
  }, py::arg("out"), py::arg("microseconds"), py::arg("blocks"), py::arg("stream"), py::arg("where") = 0,
     "probe: spinning workgroups of ~120 VGPRs per wave (a stand-in for the resident pass)");
  k.def("cu_mask_stream", [](const std::vector<uint32_t>& mask) {
    hipStream_t st = nullptr;
    MCG_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()), "stream create failed");
    return reinterpret_cast<uintptr_t>(st);
  }, "probe: a raw stream restricted to the CUs set in mask (32 per word); free with stream_destroy");
  k.def("streamop_probe", []() {
    // probe (r4): do stream memory operations (hipStreamWriteValue64 / hipStreamWaitValue64, the
    // copy-engine halo's flags) work, order a NoCU copy, and survive stream capture?
    py::dict d;
    uint64_t* flag = nullptr;
    double *a = nullptr, *b = nullptr;
    MCG_HIP(hipMalloc(&flag, 64), "probe malloc failed");
    MCG_HIP(hipMalloc(&a, 1 << 20), "probe malloc failed");
    MCG_HIP(hipMalloc(&b, 1 << 20), "probe malloc failed");
    MCG_HIP(hipMemset(flag, 0, 64), "probe memset failed");
    MCG_HIP(hipMemset(a, 0x3f, 1 << 20), "probe memset failed");
    MCG_HIP(hipMemset(b, 0, 1 << 20), "probe memset failed");
    hipStream_t s1, s2;
    MCG_HIP(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking), "stream create failed");
    MCG_HIP(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking), "stream create failed");
    // a stream that never drains must not hang the probe: poll it for up to 5 s, then release the
    // wait from the host (a plain copy into the flag) and report it
    auto drain = [&](hipStream_t s, uint64_t release, const char* key) {
      const auto t0 = std::chrono::steady_clock::now();
      hipError_t q;
      while ((q = hipStreamQuery(s)) == hipErrorNotReady &&
             std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5))
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      d[key] = q == hipErrorNotReady ? -1 : (int)q;
      if (q == hipErrorNotReady) (void)hipMemcpy(flag, &release, 8, hipMemcpyHostToDevice);
    };
    // s2: write flag = 1; s1: wait flag >= 1, then copy a -> b
    d["write"] = (int)hipStreamWriteValue64(s2, flag, 1, 0);
    d["write_done"] = (int)hipStreamSynchronize(s2);
    d["wait"] = (int)hipStreamWaitValue64(s1, flag, 1, hipStreamWaitValueGte, ~0ull);
    d["copy"] = (int)hipMemcpyAsync(b, a, 1 << 20, hipMemcpyDeviceToDeviceNoCU, s1);
    drain(s1, 1, "wait_drained");
    d["sync"] = (int)hipDeviceSynchronize();
    double h = 0;
    (void)hipMemcpy(&h, b + 1000, 8, hipMemcpyDeviceToHost);
    d["copied_ok"] = h != 0.0;
    // capture: the same ops inside a graph
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    d["cap_begin"] = (int)hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal);
    d["cap_wait"] = (int)hipStreamWaitValue64(s1, flag, 2, hipStreamWaitValueGte, ~0ull);
    d["cap_copy"] = (int)hipMemcpyAsync(a, b, 1 << 20, hipMemcpyDeviceToDeviceNoCU, s1);
    d["cap_write"] = (int)hipStreamWriteValue64(s1, flag, 3, 0);
    d["cap_end"] = (int)hipStreamEndCapture(s1, &g);
    if (g) {
      d["cap_inst"] = (int)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      (void)hipStreamWriteValue64(s2, flag, 2, 0);
      (void)hipStreamSynchronize(s2);
      if (ge) {
        d["cap_launch"] = (int)hipGraphLaunch(ge, s1);
        drain(s1, 3, "cap_drained");
        d["cap_sync"] = (int)hipStreamSynchronize(s1);
        uint64_t fv = 0;
        (void)hipMemcpy(&fv, flag, 8, hipMemcpyDeviceToHost);
        d["cap_flag_after"] = (unsigned long long)fv;
        (void)hipGraphExecDestroy(ge);
      }
      (void)hipGraphDestroy(g);
    }
    (void)hipGetLastError();
    (void)hipDeviceSynchronize();
    (void)hipStreamDestroy(s1);
    (void)hipStreamDestroy(s2);
    (void)hipFree(flag);
    (void)hipFree(a);
    (void)hipFree(b);
    return d;
  }, "probe: stream memory operations (write / wait value) with a NoCU copy, eager and captured");
  k.def("memcpy_async", [](uintptr_t dst, uintptr_t src, size_t bytes, int kind, uintptr_t stream) {
    MCG_HIP(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), bytes,
                           static_cast<hipMemcpyKind>(kind), as_stream(stream)), "memcpy async failed");
  }, py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("kind"), py::arg("stream"),
     "probe: hipMemcpyAsync of kind (3 = device to device, 1024 = device to device without compute units)");
  k.def("carry3_runs", &kern::carry3_runs, py::arg("blocks"), py::arg("jobs_per_run"), py::arg("planes"), py::arg("max_chunk") = 0,
        "the 3-D plane carry's runs of planes per job column (setup's choice)");
  k.def("stream_destroy", [](uintptr_t st) { MCG_HIP(hipStreamDestroy(reinterpret_cast<hipStream_t>(st)), "stream destroy failed"); });
  k.attr("TILE_ROWS") = kTileRows;
}
