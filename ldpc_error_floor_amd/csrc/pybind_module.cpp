// pybind_module.cpp — thin pybind11 binding over the C ABI (include/ldpc_nms.h).
// Device buffers cross as integer addresses (torch tensor .data_ptr()), streams as the
// integer hipStream_t handle; no torch or HIP types appear here.  Status < 0 raises
// RuntimeError; decode releases the GIL.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "ldpc_nms.h"

namespace py = pybind11;

static void check(int st, const char* what) {
    if (st < 0)
        throw std::runtime_error(std::string(what) + ": " + ldpc_status_string(st) + " (" +
                                 std::to_string(st) + ")");
}

struct Graph {
    ldpc_graph* h = nullptr;
    explicit Graph(py::array_t<int32_t, py::array::c_style | py::array::forcecast> proto, int z,
                   int device) {
        if (proto.ndim() != 2) throw std::invalid_argument("proto must be 2-D");
        check(ldpc_graph_create(proto.data(), (int32_t)proto.shape(0), (int32_t)proto.shape(1), z,
                                device, &h),
              "ldpc_graph_create");
    }
    ~Graph() {
        if (h) ldpc_graph_destroy(h);
    }
    py::tuple query() const {
        int32_t d[8];
        check(ldpc_graph_query(h, d), "ldpc_graph_query");
        return py::make_tuple(d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7]);
    }
    void set_weights(py::array_t<float, py::array::c_style | py::array::forcecast> alpha,
                     py::object alpha_ucn,
                     py::array_t<float, py::array::c_style | py::array::forcecast> beta) {
        if (alpha.ndim() != 2 || beta.ndim() != 2 || alpha.shape(0) != beta.shape(0))
            throw std::invalid_argument("alpha [T,E] and beta [T,N] required");
        const float* u = nullptr;
        py::array_t<float, py::array::c_style | py::array::forcecast> ua;
        if (!alpha_ucn.is_none()) {
            ua = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(alpha_ucn);
            if (!ua || ua.ndim() != 2 || ua.shape(0) != alpha.shape(0) || ua.shape(1) != alpha.shape(1))
                throw std::invalid_argument("alpha_ucn must match alpha");
            u = ua.data();
        }
        int32_t d[8];
        check(ldpc_graph_query(h, d), "ldpc_graph_query");
        if (alpha.shape(1) != d[3] || beta.shape(1) != d[1])
            throw std::invalid_argument("weight widths must be E and N");
        check(ldpc_weights_set(h, (int32_t)alpha.shape(0), alpha.data(), u, beta.data()),
              "ldpc_weights_set");
    }
};

struct Ctx {
    ldpc_ctx* h = nullptr;
    py::object graph;   // keeps the graph alive
    Ctx(py::object g, int64_t B_max, int T_max) : graph(g) {
        Graph& gr = g.cast<Graph&>();
        check(ldpc_ctx_create(gr.h, B_max, T_max, &h), "ldpc_ctx_create");
    }
    ~Ctx() {
        if (h) ldpc_ctx_destroy(h);
    }
};

static ldpc_decode_params make_params(int T, int decoding_type, int q_bit, int target_bits,
                                      float clip, int kernel) {
    ldpc_decode_params p{};
    p.T = T;
    p.decoding_type = decoding_type;
    p.q_bit = q_bit;
    p.target_bits = target_bits;
    p.clip_llr = clip;
    p.kernel = kernel;
    p.outputs_size = (int32_t)sizeof(ldpc_decode_outputs);
    return p;
}

PYBIND11_MODULE(_ldpc_nms, m) {
    m.doc() = "pybind11 binding of the MI355X NMS LDPC decoder C ABI";
    m.def("abi_version", &ldpc_abi_version);
    py::class_<Graph>(m, "Graph")
        .def(py::init<py::array_t<int32_t, py::array::c_style | py::array::forcecast>, int, int>(),
             py::arg("proto"), py::arg("z"), py::arg("device") = 0)
        .def("query", &Graph::query)
        .def("set_weights", &Graph::set_weights, py::arg("alpha"), py::arg("alpha_ucn"),
             py::arg("beta"));
    py::class_<Ctx>(m, "Ctx").def(py::init<py::object, int64_t, int>(), py::arg("graph"),
                                  py::arg("B_max"), py::arg("T_max"));
    m.def(
        "decode",
        [](Ctx& c, uintptr_t llr, int64_t B, int T, int decoding_type, int q_bit, int target_bits,
           float clip, int kernel, uintptr_t app, uintptr_t hard, uintptr_t synd,
           uintptr_t counters, uintptr_t flags, uintptr_t stream, uintptr_t iter_wrong) {
            ldpc_decode_params p = make_params(T, decoding_type, q_bit, target_bits, clip, kernel);
            ldpc_decode_outputs o{};
            o.app_all = reinterpret_cast<float*>(app);
            o.hard_bits = reinterpret_cast<uint32_t*>(hard);
            o.synd_bits = reinterpret_cast<uint32_t*>(synd);
            o.counters = reinterpret_cast<int64_t*>(counters);
            o.frame_flags = reinterpret_cast<uint8_t*>(flags);
            o.iter_wrong = reinterpret_cast<uint32_t*>(iter_wrong);
            int st;
            {
                py::gil_scoped_release nogil;
                st = ldpc_decode(c.h, reinterpret_cast<const float*>(llr), B, &p, &o,
                                 reinterpret_cast<void*>(stream));
            }
            check(st, "ldpc_decode");
        },
        py::arg("ctx"), py::arg("llr"), py::arg("B"), py::arg("T"), py::arg("decoding_type"),
        py::arg("q_bit"), py::arg("target_bits"), py::arg("clip"), py::arg("kernel"),
        py::arg("app") = 0, py::arg("hard") = 0, py::arg("synd") = 0, py::arg("counters") = 0,
        py::arg("flags") = 0, py::arg("stream") = 0, py::arg("iter_wrong") = 0);
    m.def(
        "decode_awgn",
        [](Ctx& c, int64_t B, int T, int decoding_type, int q_bit, int target_bits, float clip,
           int kernel, double sigma, uint64_t seed, int64_t offset, int ps, int pe, int ss, int se,
           uintptr_t app, uintptr_t counters, uintptr_t flags, uintptr_t stream, uintptr_t iter_wrong) {
            ldpc_decode_params p = make_params(T, decoding_type, q_bit, target_bits, clip, kernel);
            ldpc_channel_params ch{};
            ch.sigma = sigma;
            ch.seed = seed;
            ch.offset = offset;
            ch.punct_start = ps;
            ch.punct_end = pe;
            ch.short_start = ss;
            ch.short_end = se;
            ldpc_decode_outputs o{};
            o.app_all = reinterpret_cast<float*>(app);
            o.counters = reinterpret_cast<int64_t*>(counters);
            o.frame_flags = reinterpret_cast<uint8_t*>(flags);
            o.iter_wrong = reinterpret_cast<uint32_t*>(iter_wrong);
            int st;
            {
                py::gil_scoped_release nogil;
                st = ldpc_decode_awgn(c.h, B, &p, &ch, &o, reinterpret_cast<void*>(stream));
            }
            check(st, "ldpc_decode_awgn");
        },
        py::arg("ctx"), py::arg("B"), py::arg("T"), py::arg("decoding_type"), py::arg("q_bit"),
        py::arg("target_bits"), py::arg("clip"), py::arg("kernel"), py::arg("sigma"),
        py::arg("seed"), py::arg("offset"), py::arg("punct_start"), py::arg("punct_end"),
        py::arg("short_start"), py::arg("short_end"), py::arg("app") = 0, py::arg("counters") = 0,
        py::arg("flags") = 0, py::arg("stream") = 0, py::arg("iter_wrong") = 0);
    m.def(
        "channel_awgn",
        [](uintptr_t llr, int64_t B, int n_vars, double sigma, uint64_t seed, int64_t offset,
           int decoding_type, int q_bit, int ps, int pe, int ss, int se, float clip,
           uintptr_t stream) {
            int st;
            {
                py::gil_scoped_release nogil;
                st = ldpc_channel_awgn(reinterpret_cast<float*>(llr), B, n_vars, sigma, seed, offset,
                                       decoding_type, q_bit, ps, pe, ss, se, clip,
                                       reinterpret_cast<void*>(stream));
            }
            check(st, "ldpc_channel_awgn");
        },
        py::arg("llr"), py::arg("B"), py::arg("n_vars"), py::arg("sigma"), py::arg("seed"),
        py::arg("offset"), py::arg("decoding_type"), py::arg("q_bit"), py::arg("punct_start"),
        py::arg("punct_end"), py::arg("short_start"), py::arg("short_end"), py::arg("clip"),
        py::arg("stream") = 0);
    m.def(
        "channel_awgn_rows",
        [](uintptr_t rows, uintptr_t idx, int64_t n, int n_vars, double sigma, uint64_t seed,
           int64_t offset, int decoding_type, int q_bit, int ps, int pe, int ss, int se, float clip,
           uintptr_t stream) {
            check(ldpc_channel_awgn_rows(reinterpret_cast<float*>(rows), reinterpret_cast<const int64_t*>(idx),
                                         n, n_vars, sigma, seed, offset, decoding_type, q_bit, ps, pe,
                                         ss, se, clip, reinterpret_cast<void*>(stream)),
                  "ldpc_channel_awgn_rows");
        },
        py::arg("rows"), py::arg("idx"), py::arg("n"), py::arg("n_vars"), py::arg("sigma"),
        py::arg("seed"), py::arg("offset"), py::arg("decoding_type"), py::arg("q_bit"),
        py::arg("punct_start"), py::arg("punct_end"), py::arg("short_start"), py::arg("short_end"),
        py::arg("clip"), py::arg("stream") = 0);
    m.def(
        "collect_frames",
        [](uintptr_t flags, int64_t B, uint32_t mask, uint32_t want, uintptr_t idx, int64_t cap,
           uintptr_t count, uintptr_t stream) {
            check(ldpc_collect_frames(reinterpret_cast<const uint8_t*>(flags), B, mask, want,
                                      reinterpret_cast<int64_t*>(idx), cap,
                                      reinterpret_cast<int64_t*>(count),
                                      reinterpret_cast<void*>(stream)),
                  "ldpc_collect_frames");
        },
        py::arg("flags"), py::arg("B"), py::arg("mask"), py::arg("want"), py::arg("idx"),
        py::arg("cap"), py::arg("count"), py::arg("stream") = 0);
    m.def(
        "gather_rows",
        [](uintptr_t src, int64_t n_cols, uintptr_t idx, int64_t n, uintptr_t dst, uintptr_t stream) {
            check(ldpc_gather_rows(reinterpret_cast<const float*>(src), n_cols,
                                   reinterpret_cast<const int64_t*>(idx), n,
                                   reinterpret_cast<float*>(dst), reinterpret_cast<void*>(stream)),
                  "ldpc_gather_rows");
        },
        py::arg("src"), py::arg("n_cols"), py::arg("idx"), py::arg("n"), py::arg("dst"),
        py::arg("stream") = 0);
    m.def(
        "kernel_info",
        [](Ctx& c, int T, int decoding_type, int q_bit, int target_bits, int kernel, float clip) {
            ldpc_decode_params p = make_params(T, decoding_type, q_bit, target_bits, clip, kernel);
            int64_t bytes = 0;
            char name[64] = {0};
            check(ldpc_kernel_info(c.h, &p, &bytes, name, 64), "ldpc_kernel_info");
            return py::make_tuple(bytes, std::string(name));
        },
        py::arg("ctx"), py::arg("T"), py::arg("decoding_type"), py::arg("q_bit"),
        py::arg("target_bits"), py::arg("kernel"), py::arg("clip_llr") = 20.0f);
    m.def(
        "awgn_in_kernel",
        [](Ctx& c, int T, int decoding_type, int q_bit, int target_bits, int kernel, float clip,
           bool has_short, bool app) {
            ldpc_decode_params p = make_params(T, decoding_type, q_bit, target_bits, clip, kernel);
            const int r = ldpc_awgn_in_kernel(c.h, &p, has_short ? 1 : 0, app ? 1 : 0);
            check(r < 0 ? r : 0, "ldpc_awgn_in_kernel");
            return r == 1;
        },
        py::arg("ctx"), py::arg("T"), py::arg("decoding_type"), py::arg("q_bit"),
        py::arg("target_bits"), py::arg("kernel"), py::arg("clip_llr") = 20.0f,
        py::arg("has_short") = false, py::arg("app") = false);
    m.def(
        "last_kernel",
        [](Ctx& c) {
            char name[64] = {0};
            check(ldpc_ctx_last_kernel(c.h, name, 64), "ldpc_ctx_last_kernel");
            return std::string(name);
        },
        py::arg("ctx"));
    m.def(
        "format_uncor_rows",
        [](py::array_t<float, py::array::c_style | py::array::forcecast> rows) {
            if (rows.ndim() != 2 || rows.shape(1) <= 0)
                throw std::invalid_argument("rows must be [n, n_cols] with n_cols > 0");
            const int64_t n = rows.shape(0), nc = rows.shape(1);
            const int64_t step = std::max<int64_t>(1, (64 << 20) / LDPC_UNCOR_ROW_BOUND(nc));
            std::string out, buf;
            out.reserve((size_t)(n * (12 + 6 * nc)));
            buf.resize((size_t)(std::min(n, step) * LDPC_UNCOR_ROW_BOUND(nc)));
            {
                py::gil_scoped_release nogil;
                for (int64_t r0 = 0; r0 < n; r0 += step) {
                    const int64_t k = std::min(step, n - r0);
                    int64_t len = 0;
                    check(ldpc_format_uncor_rows(rows.data() + r0 * nc, k, nc, buf.data(),
                                                 (int64_t)buf.size(), &len),
                          "ldpc_format_uncor_rows");
                    out.append(buf.data(), (size_t)len);
                }
            }
            return py::bytes(out);
        },
        py::arg("rows"));
}
