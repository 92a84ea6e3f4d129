// Python bindings for the HIP workload kernels (raw device pointers + stream handles, so
// they work with torch tensors via .data_ptr() and without torch at all via gemm_burn).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <chrono>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace gpuexp {
bool gemm_shape_ok(int M, int N, int K);
bool gemm256_shape_ok(int M, int N, int K);
int resolve_gemm_variant(int M, int N, int K, int variant);
hipError_t launch_gemm_bf16_tn(const void* A, const void* B, void* C, int M, int N, int K, hipStream_t stream,
                               int variant);
hipError_t launch_fill_bf16(void* p, size_t n, uint32_t seed, hipStream_t stream);
hipError_t launch_stream_copy(const void* src, void* dst, size_t bytes, int blocks, hipStream_t stream);
hipError_t launch_lds_probe(float* out, int blocks, int iters, int stride, hipStream_t stream);
hipError_t launch_occupancy_hog(int kind, float* out, int blocks, double seconds, hipStream_t stream);
hipError_t launch_mfma_duty(float* out, uint64_t* counts, int blocks, double duty, double period_s, double seconds,
                            uint32_t xcc_mask, hipStream_t stream);
}  // namespace gpuexp

namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

// Separate module from the telemetry core: it links a HIP runtime, so it is imported
// only AFTER torch (when torch is used) to bind to torch's runtime — see ops/gemm.py.
PYBIND11_MODULE(_gpuexp_kernels, m) {
  m.doc() = "HIP/CDNA4 workload kernels (bf16 MFMA GEMM) for synthetic GPU pods";
  m.def("hip_device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("gemm_shape_ok", &gpuexp::gemm_shape_ok);
  m.def("gemm256_shape_ok", &gpuexp::gemm256_shape_ok);
  m.def("gemm_variant", &gpuexp::resolve_gemm_variant, py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("variant") = 0,
        "The GEMM kernel variant a gemm_bf16 call with these arguments runs (0 = auto resolved), -1 if the shape "
        "does not fit it.  Host-only: no GPU needed.");
  m.def("gemm_bf16", [](uintptr_t a, uintptr_t b, uintptr_t c, int M, int N, int K, uintptr_t stream, int variant) {
    if (!gpuexp::gemm_shape_ok(M, N, K))
      throw std::invalid_argument("gemm_bf16 needs M%128==0, N%128==0, K%64==0");
    if (variant >= 2 && !gpuexp::gemm256_shape_ok(M, N, K))
      throw std::invalid_argument("the 256x256 kernel needs M%256==0, N%256==0, K%64==0, K>=128");
    if (variant < 0 || variant > 9)
      throw std::invalid_argument("variant is 0 (auto), 1 (128x128), 2-9 (256x256 tile orders / priority / read schedules / ping-pong / 4 waves)");
    if (!a || !b || !c) throw std::invalid_argument("null pointer");
    check(gpuexp::launch_gemm_bf16_tn(reinterpret_cast<const void*>(a), reinterpret_cast<const void*>(b),
                                      reinterpret_cast<void*>(c), M, N, K, reinterpret_cast<hipStream_t>(stream),
                                      variant),
          "gemm_bf16 launch");
  }, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("stream") = 0,
     py::arg("variant") = 0,
     "C[M,N] = A[M,K] @ B[N,K]^T; bf16 row-major, fp32 accumulate (MFMA 16x16x32). variant: 0 auto, "
     "1 = 128x128 tile, 2 = 256x256 tile");
  m.def("fill_bf16", [](uintptr_t p, size_t n, uint32_t seed, uintptr_t stream) {
    check(gpuexp::launch_fill_bf16(reinterpret_cast<void*>(p), n, seed, reinterpret_cast<hipStream_t>(stream)),
          "fill_bf16 launch");
  }, py::arg("ptr"), py::arg("n"), py::arg("seed") = 1, py::arg("stream") = 0);
  // PMC calibration workloads (csrc/kernels/probe_kernels.hip)
  m.def("stream_copy", [](uintptr_t src, uintptr_t dst, size_t nbytes, int blocks, uintptr_t stream) {
    if (!src || !dst || nbytes % 16 || blocks < 1 || blocks > (1 << 20))
      throw std::invalid_argument("stream_copy needs non-null pointers, nbytes % 16 == 0, 1 <= blocks <= 2^20");
    check(gpuexp::launch_stream_copy(reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), nbytes, blocks,
                                     reinterpret_cast<hipStream_t>(stream)),
          "stream_copy launch");
  }, py::call_guard<py::gil_scoped_release>(), py::arg("src"), py::arg("dst"), py::arg("nbytes"),
     py::arg("blocks") = 4096, py::arg("stream") = 0,
     "dst[:nbytes] = src[:nbytes] (each byte read once from and written once to HBM)");
  m.def("lds_probe", [](uintptr_t out, int blocks, int iters, int stride, uintptr_t stream) {
    // `out` must hold >= blocks floats (checked by the Python wrapper)
    if (!out || blocks < 1 || blocks > (1 << 20) || iters < 1 || (stride != 1 && stride != 32))
      throw std::invalid_argument("lds_probe needs out, 1 <= blocks <= 2^20, iters >= 1, stride 1 or 32");
    check(gpuexp::launch_lds_probe(reinterpret_cast<float*>(out), blocks, iters, stride,
                                   reinterpret_cast<hipStream_t>(stream)),
          "lds_probe launch");
  }, py::call_guard<py::gil_scoped_release>(), py::arg("out"), py::arg("blocks"), py::arg("iters"),
     py::arg("stride"), py::arg("stream") = 0,
     "256-thread blocks (4 waves) of ds_read_b32 from LDS: stride 1 conflict-free, stride 32 32-way conflicts");
  m.def("mfma_duty", [](uintptr_t out, uintptr_t counts, int blocks, double duty, double period_s, double seconds,
                        uintptr_t stream, uint32_t xcc_mask) {
    // `out` >= blocks floats, `counts` >= blocks * 4 uint64 (checked by the Python wrapper)
    check(gpuexp::launch_mfma_duty(reinterpret_cast<float*>(out), reinterpret_cast<uint64_t*>(counts), blocks, duty,
                                   period_s, seconds, xcc_mask, reinterpret_cast<hipStream_t>(stream)),
          "mfma_duty launch");
  }, py::call_guard<py::gil_scoped_release>(), py::arg("out"), py::arg("counts"), py::arg("blocks"), py::arg("duty"),
     py::arg("period_s") = 0.002, py::arg("seconds") = 1.0, py::arg("stream") = 0, py::arg("xcc_mask") = 0,
     "256-thread blocks alternating back-to-back v_mfma_f32_32x32x16_bf16 (duty x period) with s_sleep, for "
     "`seconds` (s_memrealtime-timed); 2 blocks per CU = 2 waves per SIMD keep the matrix cores busy `duty` of "
     "the wall time.  xcc_mask != 0: only blocks on those XCCs (HW_REG_XCC_ID) run, the rest exit at once");
  m.def("occupancy_hog", [](int kind, uintptr_t out, int blocks, double seconds, uintptr_t stream) {
    // `out` >= blocks floats (checked by the Python wrapper)
    check(gpuexp::launch_occupancy_hog(kind, reinterpret_cast<float*>(out), blocks, seconds,
                                       reinterpret_cast<hipStream_t>(stream)),
          "occupancy_hog launch");
  }, py::call_guard<py::gil_scoped_release>(), py::arg("kind"), py::arg("out"), py::arg("blocks"),
     py::arg("seconds"), py::arg("stream") = 0,
     "Blocks that hold a resource for `seconds` each: kind 0 = 1 wave + 64 KiB LDS per block (LDS-limited), "
     "kind 1 = 8 waves per block, no LDS (wave-slot-limited)");
  m.def("gemm_burn", [](int device, int M, int N, int K, double seconds, int iters_per_sync, int variant) {
    // Torch-free synthetic GEMM pod: keeps one GPU busy for `seconds` and reports the
    // achieved bf16 TFLOP/s (random operands).
    if (!gpuexp::gemm_shape_ok(M, N, K) || (variant >= 2 && !gpuexp::gemm256_shape_ok(M, N, K)))
      throw std::invalid_argument("bad GEMM shape");
    if (seconds <= 0 || seconds > 3600) throw std::invalid_argument("seconds out of range");
    double tflops = 0;
    long iters = 0;
    double elapsed = 0;
    {
      py::gil_scoped_release rel;
      check(hipSetDevice(device), "hipSetDevice");
      void *a = nullptr, *b = nullptr, *c = nullptr;
      check(hipMalloc(&a, size_t(M) * K * 2), "hipMalloc A");
      check(hipMalloc(&b, size_t(N) * K * 2), "hipMalloc B");
      check(hipMalloc(&c, size_t(M) * N * 2), "hipMalloc C");
      hipStream_t s;
      check(hipStreamCreate(&s), "hipStreamCreate");
      (void)gpuexp::launch_fill_bf16(a, size_t(M) * K, 1, s);
      (void)gpuexp::launch_fill_bf16(b, size_t(N) * K, 2, s);
      check(hipStreamSynchronize(s), "fill");
      auto t0 = std::chrono::steady_clock::now();
      int per = iters_per_sync > 0 ? iters_per_sync : 8;
      for (;;) {
        for (int i = 0; i < per; ++i) check(gpuexp::launch_gemm_bf16_tn(a, b, c, M, N, K, s, variant), "gemm");
        check(hipStreamSynchronize(s), "gemm");
        iters += per;
        elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (elapsed >= seconds) break;
      }
      tflops = 2.0 * M * N * double(K) * double(iters) / elapsed / 1e12;
      (void)hipStreamDestroy(s);
      (void)hipFree(a);
      (void)hipFree(b);
      (void)hipFree(c);
    }
    py::dict d;
    d["tflops"] = tflops;
    d["iters"] = iters;
    d["seconds"] = elapsed;
    return d;
  }, py::arg("device"), py::arg("M") = 4096, py::arg("N") = 4096, py::arg("K") = 4096, py::arg("seconds") = 1.0,
     py::arg("iters_per_sync") = 8, py::arg("variant") = 0);
}
