// ldscore_py.cpp — pybind11 module `_ldscore`, the drop-in for bayarpark/nldsc's extension of the
// same name (nldsc/ldscore/_ldscore/ldscore.cpp:17-54, stub nldsc/ldscore/_ldscore.pyi:1-25).
//
// Same classes, constructor signatures (keyword-only after `bfile`), read-write attributes and
// `calculate(params) -> LDScoreResult`; the work is done by libnldsc_amd.so through the C ABI
// in include/nldsc_ld.h, on the GPU.  There is no CPU fallback: without a HIP device
// `calculate` raises RuntimeError.
//
// Differences from the reference, all additive: the GIL is released during `calculate`;
// LDScoreParams has two extra attributes, `flags` (NLDSC_FLAG_*) and `device` (HIP ordinal,
// default from $NLDSC_DEVICE, else the current device); errors carry the engine's message.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/nldsc_ld.h"

namespace py = pybind11;

namespace {

struct LDScoreParams {  // data.h:33-65
    std::string bedfile;
    int n_snp = 0;
    int n_org = 0;
    double ld_wind = 0;
    std::vector<double> positions;
    double maf = 0;
    double std_thr = 0;
    double rsq_thr = 0;
    unsigned flags = 0;
    int device = -1;

    LDScoreParams() {
        if (const char* d = std::getenv("NLDSC_DEVICE")) device = std::atoi(d);
    }
    LDScoreParams(const std::string& bfile, int n_snp_, int n_org_, double ld_wind_, double maf_, double std_thr_,
                  double rsq_thr_, const std::vector<double>& positions_)
        : LDScoreParams() {
        bedfile = bfile;
        n_snp = n_snp_;
        n_org = n_org_;
        ld_wind = ld_wind_;
        maf = maf_;
        std_thr = std_thr_;
        rsq_thr = rsq_thr_;
        positions = positions_;
    }
};

struct LDScoreResult {  // data.h:21-31
    std::vector<double> l2, l2d, maf, residuals_std;
    std::vector<int> l2_ws, l2d_ws, l2d_wse;
};

LDScoreResult calculate(const LDScoreParams& params) {
    if (params.n_snp < 0 || (size_t)params.n_snp != params.positions.size())
        throw std::invalid_argument("positions must have n_snp elements");
    LDScoreResult res;
    const size_t n = (size_t)std::max(params.n_snp, 0);
    res.l2.assign(n, 0.0);
    res.l2d.assign(n, 0.0);
    res.maf.assign(n, 0.0);
    res.residuals_std.assign(n, 0.0);
    res.l2_ws.assign(n, 0);
    res.l2d_ws.assign(n, 0);
    res.l2d_wse.assign(n, 0);
    nldsc_ld_params p{};
    p.bedfile = params.bedfile.c_str();
    p.n_snp = params.n_snp;
    p.n_org = params.n_org;
    p.ld_wind = params.ld_wind;
    p.positions = params.positions.data();
    p.maf = params.maf;
    p.std_thr = params.std_thr;
    p.rsq_thr = params.rsq_thr;
    p.flags = params.flags;
    p.device = params.device;
    nldsc_ld_result r{res.l2.data(), res.l2d.data(), res.maf.data(), res.residuals_std.data(),
                      reinterpret_cast<int32_t*>(res.l2_ws.data()), reinterpret_cast<int32_t*>(res.l2d_ws.data()),
                      reinterpret_cast<int32_t*>(res.l2d_wse.data())};
    char err[1024] = {0};
    int rc;
    {
        py::gil_scoped_release nogil;
        rc = nldsc_ld_calculate(&p, &r, err, sizeof(err));
    }
    if (rc == NLDSC_E_BAD_MAGIC) throw std::invalid_argument(err);  // -> ValueError, as the reference
    if (rc != NLDSC_OK) throw std::runtime_error(err);
    return res;
}

}  // namespace

PYBIND11_MODULE(_ldscore, m) {
    static_assert(sizeof(int) == sizeof(int32_t), "int must be 32-bit");
    py::class_<LDScoreParams> P(m, "LDScoreParams");
    P.def(py::init());
    P.def(py::init<const std::string&, int, int, double, double, double, double, const std::vector<double>&>(),
          py::arg("bfile"), py::kw_only(), py::arg("n_snp"), py::arg("n_org"), py::arg("ld_wind"), py::arg("maf"),
          py::arg("std_thr"), py::arg("rsq_thr"), py::arg("positions"));
    P.def_readwrite("bedfile", &LDScoreParams::bedfile)
        .def_readwrite("n_snp", &LDScoreParams::n_snp)
        .def_readwrite("n_org", &LDScoreParams::n_org)
        .def_readwrite("ld_wind", &LDScoreParams::ld_wind)
        .def_readwrite("positions", &LDScoreParams::positions)
        .def_readwrite("maf", &LDScoreParams::maf)
        .def_readwrite("std_thr", &LDScoreParams::std_thr)
        .def_readwrite("rsq_thr", &LDScoreParams::rsq_thr)
        .def_readwrite("flags", &LDScoreParams::flags)
        .def_readwrite("device", &LDScoreParams::device);

    py::class_<LDScoreResult> R(m, "LDScoreResult");
    R.def(py::init());
    R.def_readwrite("l2", &LDScoreResult::l2)
        .def_readwrite("l2d", &LDScoreResult::l2d)
        .def_readwrite("maf", &LDScoreResult::maf)
        .def_readwrite("residuals_std", &LDScoreResult::residuals_std)
        .def_readwrite("l2_ws", &LDScoreResult::l2_ws)
        .def_readwrite("l2d_ws", &LDScoreResult::l2d_ws)
        .def_readwrite("l2d_wse", &LDScoreResult::l2d_wse);

    m.def("calculate", &calculate);
    m.attr("__version__") = nldsc_version();
    m.attr("FLAG_STRICT_PLINK_ORDER") = NLDSC_FLAG_STRICT_PLINK_ORDER;
    m.attr("FLAG_ADDITIVE_ONLY") = NLDSC_FLAG_ADDITIVE_ONLY;
    m.attr("FLAG_EXACT_I8") = NLDSC_FLAG_EXACT_I8;
    m.attr("FLAG_FP32") = NLDSC_FLAG_FP32;
    m.attr("FLAG_EXACT_F4") = NLDSC_FLAG_EXACT_F4;
    m.attr("FLAG_EXACT_RARE") = NLDSC_FLAG_EXACT_RARE;
}
