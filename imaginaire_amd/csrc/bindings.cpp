// Python bindings for the gfx950 kernels of imaginaire_amd.
#include <torch/extension.h>

#include <vector>

namespace iamd {
// spade_norm.hip (k1)
std::vector<at::Tensor> norm_stats(const at::Tensor& x, bool per_instance, double eps,
                                   const c10::optional<at::Tensor>& weight,
                                   const c10::optional<at::Tensor>& bias, bool partial_only,
                                   const c10::optional<at::Tensor>& running_mean,
                                   const c10::optional<at::Tensor>& running_var,
                                   const c10::optional<at::Tensor>& num_batches,
                                   double momentum);
std::vector<at::Tensor> sync_stats_merge(const at::Tensor& allst, double eps,
                                         const c10::optional<at::Tensor>& weight,
                                         const c10::optional<at::Tensor>& bias,
                                         const c10::optional<at::Tensor>& running_mean,
                                         const c10::optional<at::Tensor>& running_var,
                                         const c10::optional<at::Tensor>& num_batches,
                                         double momentum);
std::vector<at::Tensor> norm_bwd_coeffs(const at::Tensor& S1, const at::Tensor& S2,
                                        const at::Tensor& rstd,
                                        const c10::optional<at::Tensor>& weight,
                                        bool per_instance, double invM, bool need_dw,
                                        bool need_db);
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
// bias_act.hip (k2)
at::Tensor bias_act_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& bias, double slope,
                        bool inplace);
std::vector<at::Tensor> bias_act_bwd(const at::Tensor& out, const at::Tensor& dy, double slope);
// partial_conv.hip (k3)
std::vector<at::Tensor> partial_conv_renorm(const at::Tensor& raw, const at::Tensor& mask,
                                            const c10::optional<at::Tensor>& bias, int64_t kh,
                                            int64_t kw, int64_t sh, int64_t sw, int64_t ph,
                                            int64_t pw, int64_t dh, int64_t dw, double winsize,
                                            double eps);
// multi_tensor.hip (k4 / k5)
void mt_adam(const std::vector<at::Tensor>& params, const std::vector<at::Tensor>& grads,
             const std::vector<at::Tensor>& exp_avgs, const std::vector<at::Tensor>& exp_avg_sqs,
             const std::vector<at::Tensor>& shadows, double lr, double beta1, double beta2,
             double eps, int64_t step, double weight_decay, bool adamw, double grad_scale,
             const c10::optional<at::Tensor>& hyper);
at::Tensor mt_sn_sigma(const std::vector<at::Tensor>& weights, const std::vector<at::Tensor>& us,
                       const std::vector<at::Tensor>& vs);
void mt_ema(const std::vector<at::Tensor>& targets, const std::vector<at::Tensor>& sources,
            double beta, const c10::optional<at::Tensor>& sigma,
            const c10::optional<at::Tensor>& count, int64_t start);
int64_t flush_deferred_uploads();
at::Tensor mt_l1_loss(const std::vector<at::Tensor>& a, const std::vector<at::Tensor>& b,
                      const std::vector<double>& w);
std::vector<at::Tensor> mt_l1_loss_backward(const std::vector<at::Tensor>& a,
                                            const std::vector<at::Tensor>& b,
                                            const std::vector<double>& w, const at::Tensor& gout);
at::Tensor mt_gan_loss(const std::vector<at::Tensor>& xs, const std::vector<int64_t>& kinds,
                       const std::vector<double>& pa, const std::vector<double>& pb,
                       const std::vector<double>& w);
std::vector<at::Tensor> mt_gan_loss_backward(const std::vector<at::Tensor>& xs,
                                             const std::vector<int64_t>& kinds,
                                             const std::vector<double>& pa,
                                             const std::vector<double>& pb,
                                             const std::vector<double>& w, const at::Tensor& gout);
at::Tensor resize_bilinear_fwd(const at::Tensor& x, int64_t Ho, int64_t Wo, double scale_h,
                               double scale_w, bool align_corners,
                               const c10::optional<at::Tensor>& add);
at::Tensor resize_bilinear_bwd(const at::Tensor& dy, int64_t H, int64_t W, double scale_h,
                               double scale_w, bool align_corners);
at::Tensor resize_nearest_fwd(const at::Tensor& x, int64_t Ho, int64_t Wo, double scale_h,
                              double scale_w);
at::Tensor resize_nearest_bwd(const at::Tensor& dy, int64_t H, int64_t W, double scale_h,
                              double scale_w);
bool stream_capturing();
void mt_scale(const std::vector<at::Tensor>& xs, const at::Tensor& s);
at::Tensor mt_sqnorm(const std::vector<at::Tensor>& xs);
// correlation.hip (k6 correlation, k8 channelnorm)
std::vector<at::Tensor> attention_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                      double scale);
std::vector<at::Tensor> attention_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                      const at::Tensor& out, const at::Tensor& lse,
                                      const at::Tensor& dout, double scale);
void nhwc_concat_into(at::Tensor& out, const at::Tensor& a, const at::Tensor& b);
at::Tensor correlation_forward(const at::Tensor& input1, const at::Tensor& input2, int64_t pad,
                               int64_t ks, int64_t md, int64_t s1, int64_t s2);
std::vector<at::Tensor> correlation_backward(const at::Tensor& input1, const at::Tensor& input2,
                                             const at::Tensor& grad_out, int64_t pad,
                                             int64_t ks, int64_t md, int64_t s1, int64_t s2);
at::Tensor channelnorm_forward(const at::Tensor& x);
at::Tensor channelnorm_backward(const at::Tensor& x, const at::Tensor& out,
                                const at::Tensor& grad_out);
// flow_warp.hip (k9 warp, k7 resample2d)
at::Tensor flow_warp_fwd(const at::Tensor& img, const at::Tensor& flow);
std::vector<at::Tensor> flow_warp_bwd(const at::Tensor& img, const at::Tensor& flow,
                                      const at::Tensor& dout,
                                      bool need_dimg);
at::Tensor resample2d_forward(const at::Tensor& in1, const at::Tensor& flow, int64_t ks);
std::vector<at::Tensor> resample2d_backward(const at::Tensor& in1, const at::Tensor& flow,
                                            const at::Tensor& dout, int64_t ks);
// conv_mfma.hip (k10)
at::Tensor channel_softmax_fwd(const at::Tensor& x);
at::Tensor conv2d_dgrad_strided(const at::Tensor& dy, const at::Tensor& w, int64_t s, int64_t ph,
                                int64_t pw, int64_t H, int64_t W, int64_t ncv,
                                const c10::optional<at::Tensor>& ascale);
std::vector<at::Tensor> mt_conv_weight_flip_t(const std::vector<at::Tensor>& ws);
at::Tensor channel_softmax_bwd(const at::Tensor& y, const at::Tensor& dy);
at::Tensor conv2d_mfma(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                       int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh, int64_t dw,
                       double slope, int64_t nb, int64_t ncv,
                       const c10::optional<at::Tensor>& residual,
                       const c10::optional<at::Tensor>& ascale);
at::Tensor conv2d_dgrad_mfma(const at::Tensor& dy, const at::Tensor& w, int64_t ph, int64_t pw,
                             int64_t ncv, const c10::optional<at::Tensor>& ascale);
at::Tensor conv2d_wgrad_mfma(const at::Tensor& dy, const at::Tensor& x, int64_t KH, int64_t KW,
                             int64_t sh, int64_t sw, int64_t ph, int64_t pw, int64_t dh,
                             int64_t dw, int64_t out_cout, int64_t out_cin, bool out_bf16,
                             int64_t nb, int64_t variant,
                             const c10::optional<std::vector<at::Tensor>>& sn,
                             const c10::optional<at::Tensor>& dst);
bool conv2d_wgrad_v2_eligible(const at::Tensor& dy, const at::Tensor& x, int64_t KH, int64_t KW,
                              int64_t sh, int64_t sw, int64_t dh, int64_t dw, int64_t nb);
// conv_tapsplit.hip
at::Tensor conv_tap_sum(const at::Tensor& z, const c10::optional<at::Tensor>& bias, int64_t Cout,
                        int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t dh, int64_t dw);
at::Tensor conv_tap_gather(const at::Tensor& dy, int64_t Cz, int64_t KH, int64_t KW, int64_t ph,
                           int64_t pw, int64_t dh, int64_t dw, int64_t H, int64_t W);
// pool.hip
at::Tensor max_pool_nhwc_fwd(const at::Tensor& x, int64_t kh, int64_t kw);
at::Tensor max_pool_nhwc_bwd(const at::Tensor& x, const at::Tensor& dy, int64_t kh, int64_t kw);
at::Tensor avg_pool_nhwc_fwd(const at::Tensor& x, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                             int64_t ph, int64_t pw, bool include_pad);
at::Tensor avg_pool_nhwc_bwd(const at::Tensor& dy, int64_t H, int64_t W, int64_t kh, int64_t kw,
                             int64_t sh, int64_t sw, int64_t ph, int64_t pw, bool include_pad);
// conv_aux.hip
at::Tensor pad_channels_cast(const at::Tensor& x, int64_t Cp, at::ScalarType dtype);
void conv_phase_scatter(const at::Tensor& src, at::Tensor& dst, int64_t s, int64_t ry, int64_t rx,
                        int64_t i0, int64_t j0, int64_t Qy, int64_t Qx);
at::Tensor conv_weight_flip_t(const at::Tensor& w, int64_t s, int64_t qy, int64_t qx,
                              int64_t nb);
std::vector<at::Tensor> conv_weight_phase_flip(const at::Tensor& w, int64_t s);
void lds_poison(int64_t blocks);
at::Tensor im2col_pack(const at::Tensor& x, int64_t KH, int64_t KW, int64_t sh, int64_t sw,
                       int64_t ph, int64_t pw, int64_t dh, int64_t dw, int64_t Kp);

int64_t conv_last_variant();
at::Tensor pad_nhwc_fwd(const at::Tensor& x, int64_t pl, int64_t pr, int64_t pt, int64_t pb,
                        int64_t mode);
at::Tensor pad_nhwc_bwd(const at::Tensor& dy, int64_t H, int64_t W, int64_t pl, int64_t pr,
                        int64_t pt, int64_t pb, int64_t mode);
at::Tensor sn_dot_partials(const at::Tensor& dx, const at::Tensor& x, const at::Tensor& sigma);
at::Tensor wgrad_finalize(const at::Tensor& part, int64_t S, int64_t Cop, int64_t Cip,
                          int64_t Cout, int64_t Cin, int64_t KH, int64_t KW,
                          at::ScalarType dtype, const c10::optional<at::Tensor>& dst);
at::Tensor sn_scale_backward(const at::Tensor& grad_in, const at::Tensor& weight,
                             const at::Tensor& u, const at::Tensor& v, const at::Tensor& sigma,
                             const c10::optional<at::Tensor>& shadow,
                             const c10::optional<at::Tensor>& dst);
void register_lmdb(pybind11::module_& m);
void profile_marker(int64_t tag);
std::vector<at::Tensor> mt_sn_scale_cast(const std::vector<at::Tensor>& weights,
                                         const at::Tensor& sigma,
                                         const std::vector<at::Tensor>& shadows,
                                         int64_t shadow_mode);
at::Tensor mt_sn_power(const std::vector<at::Tensor>& weights, const std::vector<at::Tensor>& us,
                       const std::vector<at::Tensor>& vs, bool update, double eps,
                       const std::vector<at::Tensor>& shadows);
}  // namespace iamd

namespace iamd {
at::Tensor rccl_unique_id();
int64_t rccl_comm_init(const at::Tensor& uid, int64_t rank, int64_t world);
void rccl_comm_destroy(int64_t h);
void rccl_all_reduce(const at::Tensor& t, int64_t h, int64_t op);
void rccl_all_gather(const at::Tensor& out, const at::Tensor& in, int64_t h);
}  // namespace iamd

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "imaginaire_amd gfx950 HIP kernels";
  iamd::register_lmdb(m);
  m.def("mt_sn_power", &iamd::mt_sn_power, "batched spectral-norm power iteration (k5b)",
        py::arg("weights"), py::arg("us"), py::arg("vs"), py::arg("update"), py::arg("eps"),
        py::arg("shadows") = std::vector<at::Tensor>());
  m.def("mt_sn_scale_cast", &iamd::mt_sn_scale_cast,
        "batched W/sigma -> bf16 (k5c); shadow_mode 1 reads bf16 copies of W, 2 writes them",
        py::arg("weights"), py::arg("sigma"), py::arg("shadows") = std::vector<at::Tensor>(),
        py::arg("shadow_mode") = 0);
  m.def("profile_marker", &iamd::profile_marker, "named no-op kernel for trace phase splits");
  m.def("rccl_unique_id", &iamd::rccl_unique_id, "RCCL unique id (128-byte CPU tensor)");
  m.def("rccl_comm_init", &iamd::rccl_comm_init, "join an RCCL communicator; returns a handle");
  m.def("rccl_comm_destroy", &iamd::rccl_comm_destroy, "destroy a native RCCL communicator");
  m.def("rccl_all_reduce", &iamd::rccl_all_reduce,
        "in-place all-reduce on the current stream (0 sum, 1 avg, 2 max), capturable");
  m.def("rccl_all_gather", &iamd::rccl_all_gather,
        "all-gather into a flat rank-major tensor on the current stream, capturable");
  m.def("conv2d_mfma", &iamd::conv2d_mfma, "MFMA implicit-GEMM NHWC conv + bias + act (k10)",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("sh"), py::arg("sw"), py::arg("ph"),
        py::arg("pw"), py::arg("dh"), py::arg("dw"), py::arg("slope"), py::arg("nb") = 1,
        py::arg("ncv") = -1, py::arg("residual") = py::none(), py::arg("ascale") = py::none());
  m.def("conv2d_dgrad_mfma", &iamd::conv2d_dgrad_mfma,
        "stride-1 conv data gradient from the forward weight (k10 v4 transposed-weight path)",
        py::arg("dy"), py::arg("w"), py::arg("ph"), py::arg("pw"), py::arg("ncv") = -1,
        py::arg("ascale") = py::none());
  m.def("sn_dot_partials", &iamd::sn_dot_partials,
        "sigma * <dx, x> as partial sums: <G, W> of a spectrally normalised conv (k11 SN)",
        py::arg("dx"), py::arg("x"), py::arg("sigma"));
  m.def("conv2d_wgrad_mfma", &iamd::conv2d_wgrad_mfma, "MFMA conv weight gradient (k11)",
        py::arg("dy"), py::arg("x"), py::arg("KH"), py::arg("KW"), py::arg("sh"), py::arg("sw"),
        py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"), py::arg("out_cout") = -1,
        py::arg("out_cin") = -1, py::arg("out_bf16") = false, py::arg("nb") = 1,
        py::arg("variant") = 0, py::arg("sn") = py::none(), py::arg("dst") = py::none());
  m.def("conv2d_wgrad_v2_eligible", &iamd::conv2d_wgrad_v2_eligible,
        "whether the k11 v2 (one wave per SIMD) kernel can run this weight gradient",
        py::arg("dy"), py::arg("x"), py::arg("KH"), py::arg("KW"), py::arg("sh"), py::arg("sw"),
        py::arg("dh"), py::arg("dw"), py::arg("nb") = 1);
  m.def("channel_softmax_fwd", &iamd::channel_softmax_fwd,
        "softmax over the channels of a channels-last bf16 tensor (k15)");
  m.def("channel_softmax_bwd", &iamd::channel_softmax_bwd, "k15 backward: y * (dy - sum(dy y))");
  m.def("mt_conv_weight_flip_t", &iamd::mt_conv_weight_flip_t,
        "flipped, transposed (dgrad) copies of many conv weights in one launch");
  m.def("conv2d_dgrad_strided", &iamd::conv2d_dgrad_strided,
        "strided-conv data gradient: all s*s phase convs in one k10 launch, stored in place",
        py::arg("dy"), py::arg("w"), py::arg("s"), py::arg("ph"), py::arg("pw"), py::arg("H"),
        py::arg("W"), py::arg("ncv") = -1, py::arg("ascale") = py::none());
  m.def("conv_tap_sum", &iamd::conv_tap_sum, "tap-split conv: sum of per-tap partials (+bias)");
  m.def("conv_tap_gather", &iamd::conv_tap_gather, "tap-split conv backward: dy -> per-tap dZ");
  m.def("conv_phase_scatter", &iamd::conv_phase_scatter,
        "strided-conv dgrad: one phase conv output into its parity sub-grid of dx");
  m.def("pad_channels_cast", &iamd::pad_channels_cast,
        "zero-padded channel copy + dtype cast into a channels-last tensor");
  m.def("max_pool_nhwc_fwd", &iamd::max_pool_nhwc_fwd,
        "k14 NHWC max pool, kernel == stride, no padding");
  m.def("max_pool_nhwc_bwd", &iamd::max_pool_nhwc_bwd,
        "k14 NHWC max pool backward (argmax recomputed from the input)");
  m.def("avg_pool_nhwc_fwd", &iamd::avg_pool_nhwc_fwd, "NHWC average pooling (k14)");
  m.def("avg_pool_nhwc_bwd", &iamd::avg_pool_nhwc_bwd, "k14 backward (gather)");
  m.def("pad_nhwc_fwd", &iamd::pad_nhwc_fwd, "NHWC reflect / replicate padding");
  m.def("pad_nhwc_bwd", &iamd::pad_nhwc_bwd, "NHWC reflect / replicate padding backward (gather)");
  m.def("conv_weight_flip_t", &iamd::conv_weight_flip_t,
        "flipped, in/out-transposed channels-last conv weight (dgrad-as-conv); s/qy/qx select "
        "the taps of one stride-s phase; nb per-sample weights", py::arg("w"), py::arg("s") = 1,
        py::arg("qy") = 0, py::arg("qx") = 0, py::arg("nb") = 1);
  m.def("conv_last_variant", &iamd::conv_last_variant,
        "k10 tile of the last conv2d_mfma launch on this thread (1-5, 6 = row-window)");
  m.def("im2col_pack", &iamd::im2col_pack,
        "tap-packed [M][Kp] operand of a thin-input (Cin <= 16) conv (bf16, channels-last)");
  m.def("lds_poison", &iamd::lds_poison,
        "test support: fill every CU's LDS with NaN bits (finds reads of never-written LDS)",
        py::arg("blocks") = 2048);
  m.def("conv_weight_phase_flip", &iamd::conv_weight_phase_flip,
        "all s*s phase weights conv_weight_flip_t(w, s, qy, qx) of a stride-s conv in one launch");
  m.def("sn_scale_backward", &iamd::sn_scale_backward, "spectral-norm W/sigma backward (k5d)",
        py::arg("grad"), py::arg("weight"), py::arg("u"), py::arg("v"), py::arg("sigma"),
        py::arg("shadow") = c10::optional<at::Tensor>(),
        py::arg("dst") = c10::optional<at::Tensor>());
  m.def("sync_stats_merge", &iamd::sync_stats_merge,
        "sync-BN: merge gathered per-rank (count, mean, var) rows + finalize (k1)",
        py::arg("allst"), py::arg("eps"), py::arg("weight") = py::none(),
        py::arg("bias") = py::none(), py::arg("running_mean") = py::none(),
        py::arg("running_var") = py::none(), py::arg("num_batches") = py::none(),
        py::arg("momentum") = 0.0);
  m.def("norm_stats", &iamd::norm_stats, "per-(group,channel) statistics (k1)",
        py::arg("x"), py::arg("per_instance"), py::arg("eps"), py::arg("weight"),
        py::arg("bias"), py::arg("partial_only"), py::arg("running_mean") = py::none(),
        py::arg("running_var") = py::none(), py::arg("num_batches") = py::none(),
        py::arg("momentum") = 0.0);
  m.def("norm_bwd_coeffs", &iamd::norm_bwd_coeffs, "k1 backward coefficients from the sums");
  m.def("norm_apply", &iamd::norm_apply, "norm + SPADE modulation + activation (k1 fwd)");
  m.def("norm_bwd_reduce", &iamd::norm_bwd_reduce, "k1 backward reduction");
  m.def("norm_bwd_apply", &iamd::norm_bwd_apply, "k1 backward dx");
  m.def("bias_act_fwd", &iamd::bias_act_fwd, "bias + activation epilogue (k2)");
  m.def("bias_act_bwd", &iamd::bias_act_bwd, "k2 backward: dx and dbias");
  m.def("partial_conv_renorm", &iamd::partial_conv_renorm, "partial conv mask/renorm (k3)");
  m.def("mt_adam", &iamd::mt_adam, "multi-tensor Adam/AdamW (k4)", py::arg("params"),
        py::arg("grads"), py::arg("exp_avgs"), py::arg("exp_avg_sqs"), py::arg("shadows"),
        py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"), py::arg("step"),
        py::arg("weight_decay"), py::arg("adamw"), py::arg("grad_scale"),
        py::arg("hyper") = py::none());
  m.def("stream_capturing", &iamd::stream_capturing,
        "true while the current HIP stream is being captured into a graph");
  m.def("flush_deferred_uploads", &iamd::flush_deferred_uploads,
        "copy the device tables created during a hipGraph capture (call after capture)");
  m.def("mt_sn_sigma", &iamd::mt_sn_sigma, "multi-tensor spectral-norm sigma (k5)");
  m.def("mt_ema", &iamd::mt_ema, "multi-tensor EMA with SN absorption (k5)",
        py::arg("targets"), py::arg("sources"), py::arg("beta"), py::arg("sigma") = py::none(),
        py::arg("count") = py::none(), py::arg("start") = 0);
  m.def("mt_scale", &iamd::mt_scale, "multi-tensor scale");
  m.def("mt_sqnorm", &iamd::mt_sqnorm, "multi-tensor squared L2 norm");
  m.def("mt_l1_loss", &iamd::mt_l1_loss, "multi-tensor weighted L1 loss (k13)");
  m.def("mt_l1_loss_backward", &iamd::mt_l1_loss_backward, "k13 backward");
  m.def("mt_gan_loss", &iamd::mt_gan_loss, "multi-tensor GAN loss over D outputs (k13b)");
  m.def("mt_gan_loss_backward", &iamd::mt_gan_loss_backward, "k13b backward");
  m.def("resize_bilinear_fwd", &iamd::resize_bilinear_fwd,
        "NHWC bilinear resize (+ residual) (k12)");
  m.def("resize_bilinear_bwd", &iamd::resize_bilinear_bwd, "k12 backward (gather)");
  m.def("resize_nearest_fwd", &iamd::resize_nearest_fwd, "NHWC nearest resize (k12)");
  m.def("resize_nearest_bwd", &iamd::resize_nearest_bwd, "k12 nearest backward (gather)");
  m.def("flow_warp_fwd", &iamd::flow_warp_fwd, "bilinear flow warp, border (k9)");
  m.def("flow_warp_bwd", &iamd::flow_warp_bwd, "k9 backward", py::arg("img"), py::arg("flow"),
        py::arg("dout"), py::arg("need_dimg") = true);
  m.def("resample2d_forward", &iamd::resample2d_forward, "FlowNet2 Resample2d (k7)");
  m.def("resample2d_backward", &iamd::resample2d_backward, "k7 backward");
  m.def("attention_fwd", &iamd::attention_fwd,
        "fused attention forward (k16): (softmax(scale q k^T) v, log2-domain lse)");
  m.def("attention_bwd", &iamd::attention_bwd, "fused attention backward (k16): (dq, dk, dv)");
  m.def("nhwc_concat_into", &iamd::nhwc_concat_into,
        "out = cat(a, b, zeros) along channels, NHWC (discriminator inputs)");
  m.def("correlation_forward", &iamd::correlation_forward, "FlowNet correlation (k6)");
  m.def("correlation_backward", &iamd::correlation_backward, "k6 backward");
  m.def("channelnorm_forward", &iamd::channelnorm_forward, "channel L2 norm (k8)");
  m.def("channelnorm_backward", &iamd::channelnorm_backward, "k8 backward");
}
