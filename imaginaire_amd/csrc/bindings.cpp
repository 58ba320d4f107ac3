// Python bindings for the gfx950 kernels of imaginaire_amd.
#include <torch/extension.h>

#include <vector>

namespace iamd {
// spade_norm.hip (k1)
std::vector<at::Tensor> norm_stats(const at::Tensor& x, bool per_instance, double eps,
                                   const c10::optional<at::Tensor>& weight,
                                   const c10::optional<at::Tensor>& bias, bool partial_only);
at::Tensor norm_apply(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift,
                      const c10::optional<at::Tensor>& gamma,
                      const c10::optional<at::Tensor>& beta, double slope);
std::vector<at::Tensor> norm_bwd_reduce(const at::Tensor& x, const at::Tensor& dout,
                                        const at::Tensor& scale, const at::Tensor& shift,
                                        const at::Tensor& mean, const at::Tensor& rstd,
                                        const c10::optional<at::Tensor>& gamma,
                                        const c10::optional<at::Tensor>& beta,
                                        const c10::optional<at::Tensor>& dgamma,
                                        const c10::optional<at::Tensor>& dbeta, double slope);
at::Tensor norm_bwd_apply(const at::Tensor& x, const at::Tensor& dout, const at::Tensor& scale,
                          const at::Tensor& shift, const at::Tensor& mean, const at::Tensor& rstd,
                          const at::Tensor& k1, const at::Tensor& k2, const at::Tensor& k3,
                          const c10::optional<at::Tensor>& gamma,
                          const c10::optional<at::Tensor>& beta, double slope);
}  // namespace iamd

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "imaginaire_amd gfx950 HIP kernels";
  m.def("norm_stats", &iamd::norm_stats, "per-(group,channel) statistics (k1)");
  m.def("norm_apply", &iamd::norm_apply, "norm + SPADE modulation + activation (k1 fwd)");
  m.def("norm_bwd_reduce", &iamd::norm_bwd_reduce, "k1 backward reduction");
  m.def("norm_bwd_apply", &iamd::norm_bwd_apply, "k1 backward dx");
}
