/*
 * vd_capi.h -- C-ABI of the MI355X-native Viterbi decoder (K=7, R=1/2, polynomials 0171/0133).
 *
 * This is the drop-in boundary for the reference's decode path
 * (alireza-md93/GPU-Accelerated-Viterbi-Decoder, class ViterbiCUDA<options>, src/viterbi/viterbi.h:43-152
 * and src/viterbi/viterbi.cu:10-139,210-262).  Plain pointers and sizes only: no HIP, CUDA or torch
 * types cross it.  include/viterbi.h rebuilds ViterbiCUDA<options> on top of these entry points;
 * INTEGRATION.md shows the bindings (C++ header, ctypes) a maintainer adds.
 *
 * Option bitmask: identical encoding to the reference (viterbi.h:7-20):
 *   channel  bits 0-3 : HARD=0 SOFT4=1 SOFT8=2 SOFT16=3 FP32=4
 *   metric   bits 4-7 : M_B32=0x00 M_B16=0x10 M_FP16=0x20
 *   output   bits 8-11: O_B32=0x000 O_B16=0x100
 *   compMode bits 12-15: REG=0x0000 DPX=0x1000  (DPX decodes identically to REG: the reference never
 *                        forwards compMode to its ACS, viterbi.cu:181,192,204)
 *
 * Status codes: every entry point that can fail returns an int (VD_OK = 0, negative on error) and
 * records a message readable with vd_last_error().  The header-only ViterbiCUDA wrapper maps a
 * non-zero status to stderr + exit(EXIT_FAILURE), the reference's HANDLE_ERROR behaviour
 * (gpuerrors.h:8-17).
 */
#ifndef VD_CAPI_H
#define VD_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VD_OK 0
#define VD_ERR_OPTIONS (-1)   /* option combination disabled by OptionsValid (viterbi.h:22-41) */
#define VD_ERR_ARG (-2)       /* null handle/pointer, or inputNum too small (< 128 encoded values) */
#define VD_ERR_DEVICE (-3)    /* HIP runtime error (message in vd_last_error) */
#define VD_ERR_NOMEM (-4)     /* device or pinned allocation failed */
#define VD_ERR_NOKERNEL (-5)  /* the gfx950 code object is missing from this build */

typedef struct vd_decoder vd_decoder;

/* ---- option / size helpers (replace ViterbiCUDA::getInputSize/getMessageLen/getOutputSize,
 *      viterbi.cu:63-92; sizes in bytes except vd_message_len, which is in decoded bits) ---- */

/* 1 when OptionsValid<options>::value is true (viterbi.h:22-41), else 0 */
int vd_options_valid(int options);
/* bytes of packed channel input for inputNum encoded values (getInputSize, viterbi.cu:63-84) */
size_t vd_input_size(int options, size_t inputNum);
/* decoded bits produced (getMessageLen, viterbi.cu:86-88); 0 when inputNum < 128 */
size_t vd_message_len(int options, size_t inputNum);
/* bytes of decoded output (getOutputSize, viterbi.cu:90-92) */
size_t vd_output_size(int options, size_t inputNum);
/* number of independent stream chunks the decode is partitioned into (6400, viterbi.cu:19) */
int vd_num_chunks(void);

/* ---- decoder objects (replace ViterbiCUDA() / ViterbiCUDA(size_t) / ~ViterbiCUDA,
 *      viterbi.cu:23-42,44-61) ---- */

/* Create a decoder for `options` on HIP device `device` (the reference hard-codes device 0,
 * viterbi.cu:132-139).  preallocInputNum > 0 reserves device buffers for that many encoded values,
 * so later runs of that size or smaller allocate nothing (the reference's pre-allocating
 * constructor, with the leak of viterbi.cu:31-36 fixed). */
int vd_create(int options, size_t preallocInputNum, int device, vd_decoder** out);
int vd_destroy(vd_decoder* dec);

/* Blocking host-to-host decode (replaces ViterbiCUDA::run, viterbi.cu:210-238): copies
 * vd_input_size(options, inputNum) bytes from input_h, decodes, copies vd_output_size bytes to
 * output_h.  kernel_ms (optional) receives the decode-kernel time in ms measured with HIP events,
 * the same scope as the reference's kernelTime (viterbi.cu:224-232). */
int vd_run(vd_decoder* dec, const void* input_h, void* output_h, size_t inputNum, float* kernel_ms);

/* Asynchronous device-to-device decode on `stream` (a hipStream_t passed as void*, NULL = the
 * null stream).  input_d / output_d are device pointers on the decoder's device, sized as above.
 * No allocation, no synchronisation: safe to capture in a hipGraph.  The stream (for NULL: the calling
 * thread's current device) must belong to the decoder's device, else VD_ERR_ARG.  Launches on any
 * number of streams may run concurrently: no launch shares device scratch with another. */
int vd_run_device(vd_decoder* dec, const void* input_d, void* output_d, size_t inputNum, void* stream);

/* nbatch independent batches of inputNum encoded values each in ONE launch (new; for batched callers):
 * batch b reads input_d + b * input_stride bytes and writes output_d + b * output_stride bytes.  Inputs are
 * only read, so input_stride is free (0: every batch decodes the same input; smaller than vd_input_size:
 * overlapping windows); output_stride >= vd_output_size unless nbatch == 1 (else VD_ERR_ARG: overlapping
 * outputs).  Each batch decodes exactly
 * as vd_run_device would (the reference's 6400-chunk partition per batch); one launch fills the GPU's
 * tail with the next batch's chunks.  Strides are multiples of 4 bytes; device pointers as above. */
int vd_run_device_batch(vd_decoder* dec, const void* input_d, size_t input_stride, void* output_d,
                        size_t output_stride, size_t inputNum, int nbatch, void* stream);

/* Batch sharding over several devices of one node: batch b (input_h[b] -> output_h[b],
 * each inputNum encoded values) is decoded by devices[b % ndev]; batches are independent, so the
 * result of each is identical to a single-device vd_run of that batch.  wall_ms (optional) is the
 * wall time from first H2D to last D2H. */
int vd_run_batches(int options, const void* const* input_h, void* const* output_h, size_t inputNum,
                   int nbatches, const int* devices, int ndev, float* wall_ms);

/* ---- streaming host pipeline (the reference allocates, copies and frees per call,
 *      viterbi.cu:210-238) ---- */

/* Pinned (page-locked) host buffers for full-rate PCIe copies; NULL on failure. */
void* vd_host_alloc(size_t bytes);
int vd_host_free(void* p);
/* Decode nbatches independent batches (input_h[b] -> output_h[b], inputNum encoded values each) on
 * the decoder's device.  Pinned buffers (vd_host_alloc, hipHostMalloc, hipHostRegister): the decode
 * kernels read the packed input from and write the decoded words to host memory directly over PCIe
 * (zero-copy, no staging).  Pageable buffers: H2D of batch b+1, decode of batch b and D2H of batch
 * b-1 overlap (two device buffer sets, three streams).  Each result equals vd_run of that batch.
 * wall_ms (optional): wall time of the whole call.  (vd_run also decodes zero-copy when both of its
 * host buffers are pinned.) */
int vd_run_stream(vd_decoder* dec, const void* const* input_h, void* const* output_h, int nbatches, size_t inputNum,
                  float* wall_ms);

/* ---- float channel values (the reference's SoftDecisionPacker stage, viterbiDF.h:98-167) ----
 * The reference packs float channel values on the host (quant(v*scale): HARD v > 0; SOFT4/SOFT8
 * (int)lrintf saturated to 4/8 bits; SOFT16 lrintf saturated to 16 bits; FP32 v*scale; MSB-first
 * words) and copies the packed words to the GPU.  These entry points take the floats on the device
 * instead; results are bit-identical to packing with SoftDecisionPacker(channel, scale) and then
 * decoding.  Float buffers must be 16-byte aligned; inputNum values. */

/* Pack inputNum float values into vd_input_size(options, inputNum) bytes of encPack_t words on the
 * device (a trailing partial word packs missing values as 0.0f). */
int vd_pack_device(int options, const float* llr_d, size_t inputNum, float scale, void* packed_d, void* stream);
/* Fused quantise + decode from device floats: the branch-metric table build quantises each value
 * (no packed intermediate, one kernel), every format. */
int vd_run_device_llr(vd_decoder* dec, const float* llr_d, void* output_d, size_t inputNum, float scale,
                      void* stream);
/* nbatch independent batches of inputNum device floats in one launch (as vd_run_device_batch): batch b
 * reads llr_d + b * llr_stride bytes and writes output_d + b * output_stride bytes (strides multiples
 * of 16 and 4 bytes; llr_stride free as input_stride, output_stride as vd_run_device_batch). */
int vd_run_device_llr_batch(vd_decoder* dec, const float* llr_d, size_t llr_stride, void* output_d,
                            size_t output_stride, size_t inputNum, float scale, int nbatch, void* stream);
/* Blocking host-to-host variant (H2D of the floats, fused decode, D2H); kernel_ms as in vd_run. */
int vd_run_llr(vd_decoder* dec, const float* llr_h, void* output_h, size_t inputNum, float scale, float* kernel_ms);

/* ---- the reference harness's channel source (RandBitGen | ConvolutionalEncoder | AddNoise |
 *      SoftDecisionPacker, viterbiDF.h:20-167), host and GPU ---- */

/* Host-side reference-harness generator (std::mt19937 bits + std::normal_distribution<float>
 * noise, exactly the reference pipeline's semantics, viterbiDF.h:20-167, main.cpp:131-137). */
int vd_simulate_host(int options, size_t N, float snr, uint32_t bitSeed, uint32_t noiseSeed,
                     uint8_t* bits, void* packed);
/* The reference harness's channel source on the GPU, bit-exact with vd_simulate_host for the same
 * seeds: RandBitGen(N, bitSeed) | ConvolutionalEncoder(7, 0171, 0133) | AddNoise(10^(-snr/5), noiseSeed)
 * (viterbiDF.h:20-95; std::mt19937 streams generated in parallel segments from a GF(2) jump-ahead,
 * libstdc++ uniform/normal and glibc logf restated).  bits_d: N bytes (0/1); values_d: 2N floats, the
 * AddNoise output.  Blocking (checks the polar method's sample count).  N <= 2^30. */
int vd_channel_device(size_t N, float snr, uint32_t bitSeed, uint32_t noiseSeed, uint8_t* bits_d, float* values_d,
                      void* stream);
/* vd_channel_device followed by SoftDecisionPacker(type, 40000) (viterbiDF.h:98-167): packed_d gets
 * vd_input_size(options, 2N) bytes, identical to vd_simulate_host's.  bits_d may be NULL.  N % 16 == 0. */
int vd_simulate_device(int options, size_t N, float snr, uint32_t bitSeed, uint32_t noiseSeed, uint8_t* bits_d,
                       void* packed_d, void* stream);
/* test hook: std::mt19937(seed)'s 624-word state array after n outputs (host GF(2) jump-ahead) */
int vd_mt_state_after(uint32_t seed, uint64_t n, uint32_t* state624);
/* bit-error count of a decoded buffer against the source bits (main.cpp:151-171) */
long long vd_count_errors(int options, const uint8_t* bits, size_t N, const void* decoded, size_t decodedBytes);

/* ---- runtime info ---- */
/* split launches (DESIGN.md §4 "load balance"): how many pieces of split chunks (vd_decode_tg segment
 * launches) or second chunk parts (vd_decode_pk split launches) were re-decoded on a device because their
 * speculative start had not converged at the boundary (all launches so far; decoded words are exact either
 * way).  VD_NO_SPLIT=1 in the environment (read at vd_create) disables splitting. */
int vd_split_redecodes(int device, uint64_t* count);
/* split launches (vd_decode_pk, single batches): waves on a device whose re-decode passes stopped at their cap
 * (2 P passes for P parts) with a part still differing.  The passes provably end within P (vd_kernel_pk.h
 * "Split"), so this stays 0; if it ever is not, the words of that launch may be wrong, and the blocking entry
 * points (vd_run, vd_run_llr, vd_run_stream) return VD_ERR_DEVICE after such a launch.  Callers of the
 * device-pointer entry points may check it after synchronising. */
int vd_split_cap_exits(int device, uint64_t* count);
/* LDS guard check (tests): enable != 0 makes every later launch of this decoder write guard words around
 * each wave's branch-metric table and survivor ring in LDS and count, at kernel exit, the guard words
 * found overwritten (an out-of-bounds LDS store); the count restarts at 0.  Off by default (one uniform
 * branch per wave when off).  VD_CHECK=1 in the environment turns it on at vd_create. */
int vd_set_guard_check(vd_decoder* dec, int enable);
/* guard words found overwritten since the check was enabled (synchronises the device) */
int vd_guard_violations(vd_decoder* dec, uint64_t* count);
const char* vd_last_error(void);
int vd_device_count(void);
/* the kernels an option combination can run, for profilers (static strings) */
const char* vd_kernel_name(int options);
/* the kernel and launch form this decoder takes for a decode of inputNum encoded values in nbatch batches
 * (vd_run_device: nbatch 1; vd_run_device_batch: nbatch) of packed (llr 0) or float (llr 1) input, under
 * the knobs read at vd_create (VD_NO_PK, VD_PK_SPLIT, VD_NO_SPLIT); "-" when such a decode launches
 * nothing (fewer than one output word); valid until the thread's next call */
const char* vd_decoder_kernel_name(vd_decoder* dec, size_t inputNum, int nbatch, int llr);
/* build record: "<16 hex digits of the SHA-256 of the concatenated sources> <their paths, relative to the
 * package directory>"; the Python binding refuses a library whose sources have changed since (stale build) */
const char* vd_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* VD_CAPI_H */
