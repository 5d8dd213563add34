//! `omr-gpu-sys` — thin FFI crate over `libomr_gpu.so`, the MI355X-native InstantOMR detector.
//!
//! [`ffi`] declares every entry point of `include/omr_gpu.h` (the C ABI); the safe layer mirrors
//! the `omr_core` API surface the detect path exposes (`omr_core/src/lib.rs:28-31`):
//! [`GpuDetector`] for `Detector` (`detector.rs:85-110` `new`, `:135-138` `detect`, `:169-175`
//! `detect_with_time_info`, `:223-227` `encode_pertinent_indices`, `:341-350`
//! `encode_pertinent_payloads`), [`SecretKeyPack`] for `KeyGen::generate_secret_key` /
//! `SecretKeyPack` (`key_gen/secret.rs:46-209`) with seeded streams, [`RetrievalParams`]
//! (`parameters/retrieval_params.rs:50-106`) and [`Retriever`] (`retriever.rs:188-260`).
//!
//! Differences a caller sees, all forced by determinism across GPUs and shards: keys, clues and
//! the bucket choices of `encode_pertinent_indices` come from seeded counter-based streams (the
//! reference draws from `thread_rng`), so those calls take a seed; `encode_pertinent_payloads`
//! takes the 32-byte seed the reference passes to `StdRng::from_seed` (`examples/omr.rs:197-203`)
//! and draws the same weights (`detector.rs:376-387`). `detect_batch` replaces
//! `clues.par_iter().map(|c| detector.detect(c))` (`examples/omr.rs:160-164`).
//!
//! The crate has no dependencies; `build.rs` links `libomr_gpu.so` and the HIP runtime.

use std::ffi::CStr;
use std::fmt;
use std::os::raw::{c_char, c_int, c_long, c_void};
use std::time::Duration;

/// Raw bindings of `include/omr_gpu.h`, one declaration per C entry point.
pub mod ffi {
    use super::*;

    pub type OmrStatus = c_int;
    pub const OMR_OK: OmrStatus = 0;
    pub const OMR_ERR_INVALID_ARGUMENT: OmrStatus = 1;
    pub const OMR_ERR_DEVICE: OmrStatus = 2;
    pub const OMR_ERR_OUT_OF_MEMORY: OmrStatus = 3;
    pub const OMR_ERR_NOT_INVERTIBLE: OmrStatus = 4;

    pub const OMR_N0: usize = 512;
    pub const OMR_Q0: u32 = 2048;
    pub const OMR_CLUE_COUNT: usize = 7;
    pub const OMR_Q1: u32 = 134215681;
    pub const OMR_N1: usize = 1024;
    pub const OMR_KS_DIGITS: usize = 27;
    pub const OMR_NI: usize = 670;
    pub const OMR_QI: u32 = 4096;
    pub const OMR_Q2: u64 = 1125899906826241;
    pub const OMR_N2: usize = 2048;
    pub const OMR_TRACE_STEPS: usize = 11;
    pub const OMR_TRACE_DIGITS: usize = 25;
    pub const OMR_P: u32 = 257;
    pub const OMR_PAYLOAD_LEN: usize = 612;

    #[repr(C)]
    pub struct OmrSecretKeyPack {
        _private: [u8; 0],
    }
    #[repr(C)]
    pub struct OmrCtx {
        _private: [u8; 0],
    }
    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
    pub struct OmrRetrievalParams {
        pub index_slots_per_bucket: u32,
        pub slots_per_bucket: u32,
        pub slots_per_segment: u32,
        pub segment_per_cipher: u32,
        pub max_encode_indices_cipher_count: u32,
        pub combination_count: u32,
        pub cmb_count_per_cipher: u32,
        pub cmb_cipher_count: u32,
    }
    #[repr(C)]
    #[derive(Clone, Copy, Debug)]
    pub struct OmrDetectionKeyView {
        pub bsk1: *const u32,
        pub ksk: *const u32,
        pub bsk2: *const u64,
        pub trace_key: *const u64,
    }
    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default)]
    pub struct OmrDetectTiming {
        pub total_ms: f32,
        pub first_level_ms: f32,
        pub second_level_ms: f32,
        pub trace_ms: f32,
        pub key_switch_ms: f32,
        pub messages: usize,
        pub trace_separate: c_int,
    }

    extern "C" {
        pub fn omr_last_error() -> *const c_char;
        pub fn omr_version() -> *const c_char;

        // key generation (key_gen/mod.rs:21-27, key_gen/secret.rs:46-178, clue.rs:27-34)
        pub fn omr_keygen_secret(seed: u64, out: *mut *mut OmrSecretKeyPack) -> OmrStatus;
        pub fn omr_secret_destroy(sk: *mut OmrSecretKeyPack);
        pub fn omr_secret_export(sk: *const OmrSecretKeyPack, s0: *mut u8, s1: *mut i8, s_int: *mut u8,
                                 s2: *mut i8) -> OmrStatus;
        pub fn omr_keygen_detection_key(sk: *const OmrSecretKeyPack, seed: u64, bsk1: *mut u32, ksk: *mut u32,
                                        bsk2: *mut u64, trace_key: *mut u64, nthreads: c_int) -> OmrStatus;
        pub fn omr_gen_clues(sk: *const OmrSecretKeyPack, seed: u64, first: u64, count: usize, clue_a: *mut u16,
                             clue_b: *mut u16, nthreads: c_int) -> OmrStatus;
        pub fn omr_gen_clues_device(sk: *const OmrSecretKeyPack, seed: u64, first: u64, count: usize,
                                    d_clue_a: *mut u16, d_clue_b: *mut u16, stream: *mut c_void) -> OmrStatus;
        pub fn omr_keygen_detection_key_device(sk: *const OmrSecretKeyPack, seed: u64, d_bsk1: *mut u32,
                                               d_ksk: *mut u32, d_bsk2: *mut u64, d_trace_key: *mut u64,
                                               stream: *mut c_void) -> OmrStatus;

        // retrieval layout and payload weights (retrieval_params.rs:50-106, detector.rs:376-387)
        pub fn omr_get_retrieval_params(all_payloads_count: usize, pertinent_count: usize,
                                        out: *mut OmrRetrievalParams) -> OmrStatus;
        pub fn omr_payload_weights(seed: *const u8, all_payloads_count: usize, combination_count: u32,
                                   cmb_cipher_count: u32, cmb_count_per_cipher: u32, out: *mut u16) -> OmrStatus;

        // retriever (retriever.rs:63-130, 188-260; matrix.rs:164-247)
        pub fn omr_decrypt_decode(sk: *const OmrSecretKeyPack, ct: *const u64, n: usize, out: *mut u32) -> OmrStatus;
        pub fn omr_retrieve_indices(sk: *const OmrSecretKeyPack, idx_cts: *const u64, n_ct: u32,
                                    all_payloads_count: usize, pertinent_count: usize, indices: *mut usize,
                                    cap: usize, found: *mut usize) -> OmrStatus;
        pub fn omr_retrieve_payloads(sk: *const OmrSecretKeyPack, pay_cts: *const u64, n_ct: u32,
                                     all_payloads_count: usize, combination_count: u32, weights: *const u16,
                                     indices: *const usize,
                                     n_indices: usize, payloads: *mut u16) -> OmrStatus;

        // detector (detector.rs:85-453)
        pub fn omr_ctx_create(key: *const OmrDetectionKeyView, device: c_int, out: *mut *mut OmrCtx) -> OmrStatus;
        pub fn omr_ctx_destroy(ctx: *mut OmrCtx);
        pub fn omr_detect_kernels() -> *const c_char;
        pub fn omr_ctx_set_batch(ctx: *mut OmrCtx, batch: usize) -> OmrStatus;
        pub fn omr_ctx_set_latency_threshold(ctx: *mut OmrCtx, max_messages: usize) -> OmrStatus;
        pub fn omr_ctx_set_exact_level1(ctx: *mut OmrCtx, enable: c_int) -> OmrStatus;
        pub fn omr_ctx_set_encode_chunks(ctx: *mut OmrCtx, max_chunks: usize) -> OmrStatus;
        pub fn omr_detect_batch(ctx: *mut OmrCtx, clue_a: *const u16, clue_b: *const u16, d: usize,
                                out: *mut u64) -> OmrStatus;
        pub fn omr_detect(ctx: *mut OmrCtx, clue_a: *const u16, clue_b: *const u16, out: *mut u64) -> OmrStatus;
        pub fn omr_ctx_set_coalescing(ctx: *mut OmrCtx, max_messages: usize, window_us: c_long) -> OmrStatus;
        pub fn omr_ctx_coalescing_stats(ctx: *mut OmrCtx, calls: *mut usize, launches: *mut usize) -> OmrStatus;
        pub fn omr_detect_batch_device(ctx: *mut OmrCtx, d_clue_a: *const u16, d_clue_b: *const u16, d: usize,
                                       d_out: *mut u64, hip_stream: *mut c_void) -> OmrStatus;
        pub fn omr_ctx_enable_timing(ctx: *mut OmrCtx, mode: c_int) -> OmrStatus;
        pub fn omr_last_timing(ctx: *mut OmrCtx, t: *mut OmrDetectTiming) -> OmrStatus;
        pub fn omr_detect_with_time_info(ctx: *mut OmrCtx, clue_a: *const u16, clue_b: *const u16, d: usize,
                                         out: *mut u64, t: *mut OmrDetectTiming) -> OmrStatus;
        pub fn omr_ctx_check(ctx: *mut OmrCtx, hip_stream: *mut c_void) -> OmrStatus;
        pub fn omr_ctx_set_rounding_guard(ctx: *mut OmrCtx, enable: c_int) -> OmrStatus;
        pub fn omr_ctx_rounding_margin(ctx: *mut OmrCtx, observed: *mut f64, apriori: *mut f64, kappa: *mut f64,
                                       reset: c_int) -> OmrStatus;
        pub fn omr_ctx_exactness(ctx: *mut OmrCtx, guarded: *mut c_int, breaches: *mut u64) -> OmrStatus;
        pub fn omr_fft_twiddles_dd(level: c_int, out: *mut f64) -> OmrStatus;
        pub fn omr_ctx_key_spectrum(ctx: *mut OmrCtx, level: c_int, first: usize, count: usize,
                                    out: *mut f64) -> OmrStatus;
        pub fn omr_encode_indices(ctx: *mut OmrCtx, pv: *const u64, d: usize, global_offset: usize,
                                  all_payloads_count: usize, seed: u64, ct: u32, out: *mut u64) -> OmrStatus;
        pub fn omr_encode_indices_device(ctx: *mut OmrCtx, d_pv: *const u64, d: usize, global_offset: usize,
                                         all_payloads_count: usize, seed: u64, first_ct: u32, n_ct: u32,
                                         d_out: *mut u64, hip_stream: *mut c_void) -> OmrStatus;
        pub fn omr_encode_payloads(ctx: *mut OmrCtx, pv: *const u64, payloads: *const u16, d: usize,
                                   global_offset: usize, all_payloads_count: usize, weights: *const u16, n_ct: u32,
                                   cmb_per_ct: u32, out: *mut u64) -> OmrStatus;
        pub fn omr_encode_payloads_device(ctx: *mut OmrCtx, d_pv: *const u64, d_payloads: *const u16, d: usize,
                                          global_offset: usize, all_payloads_count: usize, d_weights: *const u16,
                                          n_ct: u32, cmb_per_ct: u32, d_out: *mut u64,
                                          hip_stream: *mut c_void) -> OmrStatus;

        // stage entry points (benches/two_level_bs.rs)
        pub fn omr_first_level(ctx: *mut OmrCtx, clue_a: *const u16, clue_b: *const u16, d: usize,
                               lwe_int: *mut u32) -> OmrStatus;
        pub fn omr_blind_rotate_level1(ctx: *mut OmrCtx, lwe_a: *const u16, lwe_b: *const u16, n: usize,
                                       out: *mut u64) -> OmrStatus;
        pub fn omr_fft1_mul(ctx: *mut OmrCtx, a: *const u32, k: *const u32, n: usize, out: *mut u64) -> OmrStatus;
        pub fn omr_second_level(ctx: *mut OmrCtx, lwe_int: *const u32, n: usize, out: *mut u64) -> OmrStatus;
        pub fn omr_blind_rotate_level2(ctx: *mut OmrCtx, lwe_int: *const u32, n: usize, out: *mut u64) -> OmrStatus;
        pub fn omr_ntt(level: c_int, inverse: c_int, polys: *mut u64, n: usize, device: c_int) -> OmrStatus;
    }
}

use ffi::*;

/// A failed library call: the status code and `omr_last_error()`'s message.
#[derive(Debug, Clone)]
pub struct OmrError {
    pub status: OmrStatus,
    pub message: String,
}

impl fmt::Display for OmrError {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "omr_gpu status {}: {}", self.status, self.message)
    }
}
impl std::error::Error for OmrError {}

fn check(st: OmrStatus) -> Result<(), OmrError> {
    if st == OMR_OK {
        return Ok(());
    }
    let message = unsafe { CStr::from_ptr(omr_last_error()) }.to_string_lossy().into_owned();
    Err(OmrError { status: st, message })
}

/// `CmLweCiphertext<u16>` of one message: mask `a` (512) and the 7 bodies, values mod 2048.
#[derive(Clone)]
pub struct Clue {
    pub a: [u16; OMR_N0],
    pub b: [u16; OMR_CLUE_COUNT],
}

/// `NttRlweCiphertext<SecondLevelField>`: (a, b) in the NTT domain (include/omr_gpu.h order).
#[derive(Clone)]
pub struct NttRlwe {
    pub a: Box<[u64; OMR_N2]>,
    pub b: Box<[u64; OMR_N2]>,
}

impl NttRlwe {
    fn from_flat(v: &[u64]) -> Self {
        let mut a = Box::new([0u64; OMR_N2]);
        let mut b = Box::new([0u64; OMR_N2]);
        a.copy_from_slice(&v[..OMR_N2]);
        b.copy_from_slice(&v[OMR_N2..2 * OMR_N2]);
        NttRlwe { a, b }
    }
    fn flatten(items: &[NttRlwe]) -> Vec<u64> {
        let mut v = Vec::with_capacity(items.len() * 2 * OMR_N2);
        for c in items {
            v.extend_from_slice(&c.a[..]);
            v.extend_from_slice(&c.b[..]);
        }
        v
    }
}

/// `Payload` (payload.rs:14): 612 values, bytes stored as u16.
pub type Payload = [u16; OMR_PAYLOAD_LEN];

/// `RetrievalParams::new(257, 2048, all, pertinent, 130, 25, 2)` (retrieval_params.rs:50-106).
#[derive(Clone, Copy, Debug)]
pub struct RetrievalParams {
    pub all_payloads_count: usize,
    pub pertinent_count: usize,
    pub layout: OmrRetrievalParams,
}

impl RetrievalParams {
    pub fn new(all_payloads_count: usize, pertinent_count: usize) -> Result<Self, OmrError> {
        let mut layout = OmrRetrievalParams::default();
        check(unsafe { omr_get_retrieval_params(all_payloads_count, pertinent_count, &mut layout) })?;
        Ok(Self { all_payloads_count, pertinent_count, layout })
    }
    pub fn max_encode_indices_cipher_count(&self) -> usize {
        self.layout.max_encode_indices_cipher_count as usize
    }
    pub fn combination_count(&self) -> usize {
        self.layout.combination_count as usize
    }
    pub fn cmb_count_per_cipher(&self) -> usize {
        self.layout.cmb_count_per_cipher as usize
    }
}

/// Payload weights `StdRng::from_seed(seed)` + `Uniform<u16>(0, 257)` in the reference order
/// (detector.rs:376-387), `[cmb_cipher_count * cmb_count_per_cipher][all]`.
pub fn payload_weights(seed: &[u8; 32], rp: &RetrievalParams) -> Result<Vec<u16>, OmrError> {
    let l = rp.layout;
    let mut out = vec![0u16; (l.cmb_cipher_count * l.cmb_count_per_cipher) as usize * rp.all_payloads_count];
    check(unsafe {
        omr_payload_weights(seed.as_ptr(), rp.all_payloads_count, l.combination_count, l.cmb_cipher_count,
                            l.cmb_count_per_cipher, out.as_mut_ptr())
    })?;
    Ok(out)
}

/// Coefficient-domain evaluation keys in the include/omr_gpu.h layout (`DetectionKey`,
/// key_gen/detection.rs:9-16).
pub struct DetectionKey {
    pub bsk1: Vec<u32>,
    pub ksk: Vec<u32>,
    pub bsk2: Vec<u64>,
    pub trace_key: Vec<u64>,
}

pub const BSK1_LEN: usize = OMR_N0 * 8 * 2 * OMR_N1;
pub const KSK_LEN: usize = OMR_N1 * OMR_KS_DIGITS * (OMR_NI + 1);
pub const BSK2_LEN: usize = OMR_NI * 12 * 2 * OMR_N2;
pub const TRACE_KEY_LEN: usize = OMR_TRACE_STEPS * OMR_TRACE_DIGITS * 2 * OMR_N2;

/// `SecretKeyPack` from `KeyGen::generate_secret_key`, deterministic from a 64-bit seed.
pub struct SecretKeyPack {
    raw: *mut OmrSecretKeyPack,
}
unsafe impl Send for SecretKeyPack {}
unsafe impl Sync for SecretKeyPack {}

impl SecretKeyPack {
    pub fn generate(seed: u64) -> Result<Self, OmrError> {
        let mut raw = std::ptr::null_mut();
        check(unsafe { omr_keygen_secret(seed, &mut raw) })?;
        Ok(Self { raw })
    }
    /// `generate_detection_key` (secret.rs:118-178) on `nthreads` host threads (0: all).
    pub fn generate_detection_key(&self, seed: u64, nthreads: i32) -> Result<DetectionKey, OmrError> {
        let mut k = DetectionKey { bsk1: vec![0; BSK1_LEN], ksk: vec![0; KSK_LEN], bsk2: vec![0; BSK2_LEN],
                                   trace_key: vec![0; TRACE_KEY_LEN] };
        check(unsafe {
            omr_keygen_detection_key(self.raw, seed, k.bsk1.as_mut_ptr(), k.ksk.as_mut_ptr(), k.bsk2.as_mut_ptr(),
                                     k.trace_key.as_mut_ptr(), nthreads)
        })?;
        Ok(k)
    }
    /// `Sender::gen_clues` (sender.rs:27-32) for global message indices `first..first + count`.
    pub fn gen_clues(&self, seed: u64, first: u64, count: usize) -> Result<Vec<Clue>, OmrError> {
        let mut a = vec![0u16; count * OMR_N0];
        let mut b = vec![0u16; count * OMR_CLUE_COUNT];
        check(unsafe { omr_gen_clues(self.raw, seed, first, count, a.as_mut_ptr(), b.as_mut_ptr(), 0) })?;
        Ok((0..count)
            .map(|m| {
                let mut c = Clue { a: [0; OMR_N0], b: [0; OMR_CLUE_COUNT] };
                c.a.copy_from_slice(&a[m * OMR_N0..(m + 1) * OMR_N0]);
                c.b.copy_from_slice(&b[m * OMR_CLUE_COUNT..(m + 1) * OMR_CLUE_COUNT]);
                c
            })
            .collect())
    }
}

impl Drop for SecretKeyPack {
    fn drop(&mut self) {
        unsafe { omr_secret_destroy(self.raw) }
    }
}

/// `DetectTimeInfo` (detector.rs:51-57): summed device time per stage of a detect batch.
#[derive(Debug, Clone, Copy, Default)]
pub struct DetectTimeInfo {
    pub total_detect_time: Duration,
    /// 7 level-1 rotations + sum + key switch + modulus switch (detector.rs:183-189)
    pub total_first_level_bootstrapping_time: Duration,
    /// level-2 blind rotation (detector.rs:193-198)
    pub total_second_level_bootstrapping_time: Duration,
    /// hom_trace + NTT (detector.rs:202-209)
    pub total_trace_time: Duration,
}

impl From<OmrDetectTiming> for DetectTimeInfo {
    fn from(t: OmrDetectTiming) -> Self {
        let ms = |v: f32| Duration::from_secs_f64(f64::from(v.max(0.0)) * 1e-3);
        Self {
            total_detect_time: ms(t.total_ms),
            total_first_level_bootstrapping_time: ms(t.first_level_ms),
            total_second_level_bootstrapping_time: ms(t.second_level_ms),
            total_trace_time: ms(t.trace_ms),
        }
    }
}

/// `Detector` on one MI355X: owns the device-resident evaluation keys.
pub struct GpuDetector {
    ctx: *mut OmrCtx,
}
// Calls on one context are serialised inside the library; contexts are independent.
unsafe impl Send for GpuDetector {}
unsafe impl Sync for GpuDetector {}

impl GpuDetector {
    /// `Detector::new` (detector.rs:85-110): uploads the keys to `device` and converts them.
    pub fn new(key: &DetectionKey, device: i32) -> Result<Self, OmrError> {
        if key.bsk1.len() != BSK1_LEN || key.ksk.len() != KSK_LEN || key.bsk2.len() != BSK2_LEN
            || key.trace_key.len() != TRACE_KEY_LEN
        {
            return Err(OmrError { status: OMR_ERR_INVALID_ARGUMENT, message: "detection key sizes".into() });
        }
        let view = OmrDetectionKeyView { bsk1: key.bsk1.as_ptr(), ksk: key.ksk.as_ptr(), bsk2: key.bsk2.as_ptr(),
                                         trace_key: key.trace_key.as_ptr() };
        let mut ctx = std::ptr::null_mut();
        check(unsafe { omr_ctx_create(&view, device, &mut ctx) })?;
        Ok(Self { ctx })
    }

    /// `Detector::detect` (detector.rs:135-138): one clue set, a batch of one.
    pub fn detect(&self, clue: &Clue) -> Result<NttRlwe, OmrError> {
        // omr_detect coalesces concurrent callers (e.g. rayon's par_iter over a shared &Detector,
        // examples/omr.rs:160-164) into batched launches
        let mut out = vec![0u64; 2 * OMR_N2];
        check(unsafe { omr_detect(self.ctx, clue.a.as_ptr(), clue.b.as_ptr(), out.as_mut_ptr()) })?;
        Ok(NttRlwe::from_flat(&out))
    }

    /// `clues.par_iter().map(|c| detector.detect(c))` (examples/omr.rs:160-164) in one call.
    pub fn detect_batch(&self, clues: &[Clue]) -> Result<Vec<NttRlwe>, OmrError> {
        let d = clues.len();
        let mut a = Vec::with_capacity(d * OMR_N0);
        let mut b = Vec::with_capacity(d * OMR_CLUE_COUNT);
        for c in clues {
            a.extend_from_slice(&c.a);
            b.extend_from_slice(&c.b);
        }
        let mut out = vec![0u64; d * 2 * OMR_N2];
        check(unsafe { omr_detect_batch(self.ctx, a.as_ptr(), b.as_ptr(), d, out.as_mut_ptr()) })?;
        Ok(out.chunks_exact(2 * OMR_N2).map(NttRlwe::from_flat).collect())
    }

    /// `Detector::detect_with_time_info` (detector.rs:169-221) over a batch: detect and the stage
    /// times in one call under the context's lock (safe with concurrent callers).
    pub fn detect_with_time_info(&self, clues: &[Clue]) -> Result<(Vec<NttRlwe>, DetectTimeInfo), OmrError> {
        let d = clues.len();
        let mut a = Vec::with_capacity(d * OMR_N0);
        let mut b = Vec::with_capacity(d * OMR_CLUE_COUNT);
        for c in clues {
            a.extend_from_slice(&c.a);
            b.extend_from_slice(&c.b);
        }
        let mut out = vec![0u64; d * 2 * OMR_N2];
        let mut t = OmrDetectTiming::default();
        check(unsafe { omr_detect_with_time_info(self.ctx, a.as_ptr(), b.as_ptr(), d, out.as_mut_ptr(), &mut t) })?;
        Ok((out.chunks_exact(2 * OMR_N2).map(NttRlwe::from_flat).collect(), t.into()))
    }

    /// Waits for `hip_stream` (null = the whole device) and reports a failed earlier device
    /// call on this context (`omr_ctx_check`); callers of the device entry points use it.
    pub fn check(&self, hip_stream: *mut c_void) -> Result<(), OmrError> {
        check(unsafe { omr_ctx_check(self.ctx, hip_stream) })
    }

    /// `Detector::encode_pertinent_indices` (detector.rs:223-227) for index ciphertext `ct` of the
    /// board; the buckets come from `seed` (the reference draws them from thread_rng, :262).
    pub fn encode_pertinent_indices(&self, rp: &RetrievalParams, pertinency_vector: &[NttRlwe], seed: u64,
                                    ct: u32) -> Result<NttRlwe, OmrError> {
        self.encode_pertinent_indices_shard(rp, pertinency_vector, 0, seed, ct)
    }

    /// The same over the board's messages `global_offset..global_offset + pv.len()` (one shard of
    /// a multi-GPU job; the partial digests are summed mod q2).
    pub fn encode_pertinent_indices_shard(&self, rp: &RetrievalParams, pertinency_vector: &[NttRlwe],
                                          global_offset: usize, seed: u64, ct: u32) -> Result<NttRlwe, OmrError> {
        let pv = NttRlwe::flatten(pertinency_vector);
        let mut out = vec![0u64; 2 * OMR_N2];
        check(unsafe {
            omr_encode_indices(self.ctx, pv.as_ptr(), pertinency_vector.len(), global_offset, rp.all_payloads_count,
                               seed, ct, out.as_mut_ptr())
        })?;
        Ok(NttRlwe::from_flat(&out))
    }

    /// `Detector::encode_pertinent_payloads` (detector.rs:341-350) with the 32-byte seed of
    /// `StdRng::from_seed` (same weights; the retriever regenerates them, retriever.rs:215-240).
    pub fn encode_pertinent_payloads(&self, pertinency_vector: &[NttRlwe], payloads: &[Payload],
                                     rp: &RetrievalParams, seed: &[u8; 32]) -> Result<Vec<NttRlwe>, OmrError> {
        if payloads.len() != pertinency_vector.len() {
            return Err(OmrError { status: OMR_ERR_INVALID_ARGUMENT, message: "one payload per message".into() });
        }
        let w = payload_weights(seed, rp)?;
        let pv = NttRlwe::flatten(pertinency_vector);
        let pay: Vec<u16> = payloads.iter().flat_map(|p| p.iter().copied()).collect();
        let n_ct = rp.layout.cmb_cipher_count;
        let mut out = vec![0u64; n_ct as usize * 2 * OMR_N2];
        check(unsafe {
            omr_encode_payloads(self.ctx, pv.as_ptr(), pay.as_ptr(), pertinency_vector.len(), 0,
                                rp.all_payloads_count, w.as_ptr(), n_ct, rp.layout.cmb_count_per_cipher,
                                out.as_mut_ptr())
        })?;
        Ok(out.chunks_exact(2 * OMR_N2).map(NttRlwe::from_flat).collect())
    }

    /// Messages per internal detect chunk (0 = default).
    pub fn set_batch(&self, batch: usize) -> Result<(), OmrError> {
        check(unsafe { omr_ctx_set_batch(self.ctx, batch) })
    }

    /// At most `max_chunks` partial digests per encode ciphertext (0 = default 4,096).
    pub fn set_encode_chunks(&self, max_chunks: usize) -> Result<(), OmrError> {
        check(unsafe { omr_ctx_set_encode_chunks(self.ctx, max_chunks) })
    }

    /// Coalescing of concurrent `detect` callers (`omr_ctx_set_coalescing`): at most
    /// `max_messages` per combined launch (0 = 65,536), launching after `window_us` microseconds.
    pub fn set_coalescing(&self, max_messages: usize, window_us: i64) -> Result<(), OmrError> {
        check(unsafe { omr_ctx_set_coalescing(self.ctx, max_messages, window_us as c_long) })
    }

    /// Rounding-margin guard of the FFT external products (`omr_ctx_set_rounding_guard`).
    pub fn set_rounding_guard(&self, enable: bool) -> Result<(), OmrError> {
        check(unsafe { omr_ctx_set_rounding_guard(self.ctx, enable as c_int) })
    }

    /// (observed margins, a priori bounds) per level (`omr_ctx_rounding_margin`): a guarded run is
    /// exact when observed < 1 - apriori (and every run when apriori < 0.5).
    pub fn rounding_margin(&self, reset: bool) -> Result<([f64; 2], [f64; 2]), OmrError> {
        let (mut obs, mut apr) = ([0f64; 2], [0f64; 2]);
        check(unsafe {
            omr_ctx_rounding_margin(self.ctx, obs.as_mut_ptr(), apr.as_mut_ptr(), std::ptr::null_mut(), reset as c_int)
        })?;
        Ok((obs, apr))
    }

    /// The exactness contract (`omr_ctx_exactness`): (guarded on every launch, breaching launches)
    /// per level. A level whose a priori bound is >= 0.5 is guarded automatically; a breach on
    /// either level was re-run on the exact NTT (level 1: br1n_fallback_kernel; level 2:
    /// br2l_fallback_kernel + trace_fallback_kernel).
    pub fn exactness(&self) -> Result<([bool; 2], [u64; 2]), OmrError> {
        let (mut g, mut b) = ([0 as c_int; 2], [0u64; 2]);
        check(unsafe { omr_ctx_exactness(self.ctx, g.as_mut_ptr(), b.as_mut_ptr()) })?;
        Ok(([g[0] != 0, g[1] != 0], b))
    }

    /// Chunks of at most `max_messages` messages run the latency kernels (0 = never).
    pub fn set_latency_threshold(&self, max_messages: usize) -> Result<(), OmrError> {
        check(unsafe { omr_ctx_set_latency_threshold(self.ctx, max_messages) })
    }

    /// Level 1 on the exact modular NTT for every launch (`omr_ctx_set_exact_level1`): the
    /// reference's arithmetic, bit-identical outputs, slower.
    pub fn set_exact_level1(&self, enable: bool) -> Result<(), OmrError> {
        check(unsafe { omr_ctx_set_exact_level1(self.ctx, enable as c_int) })
    }
}

impl Drop for GpuDetector {
    fn drop(&mut self) {
        unsafe { omr_ctx_destroy(self.ctx) }
    }
}

/// `Retriever::decode_digest` (retriever.rs:188-260) under the pack's second-level key.
pub struct Retriever<'a> {
    pub params: RetrievalParams,
    pub secret: &'a SecretKeyPack,
}

impl<'a> Retriever<'a> {
    /// Sorted pertinent indices and their payloads; `seed` is the payload-weight seed.
    pub fn decode_digest(&self, indices_digest: &[NttRlwe], payloads_digest: &[NttRlwe],
                         seed: &[u8; 32]) -> Result<(Vec<usize>, Vec<Payload>), OmrError> {
        let rp = self.params;
        let idx = NttRlwe::flatten(indices_digest);
        let mut found_buf = vec![0usize; rp.pertinent_count.max(1) * 4 + 64];
        let mut found = 0usize;
        check(unsafe {
            omr_retrieve_indices(self.secret.raw, idx.as_ptr(), indices_digest.len() as u32, rp.all_payloads_count,
                                 rp.pertinent_count, found_buf.as_mut_ptr(), found_buf.len(), &mut found)
        })?;
        found_buf.truncate(found.min(found_buf.len()));
        // the board's weights and combination count, whatever the number of indices found
        // (retriever.rs:196, :215-239)
        let w = payload_weights(seed, &rp)?;
        let pay = NttRlwe::flatten(payloads_digest);
        let mut out = vec![0u16; found_buf.len() * OMR_PAYLOAD_LEN];
        check(unsafe {
            omr_retrieve_payloads(self.secret.raw, pay.as_ptr(), payloads_digest.len() as u32, rp.all_payloads_count,
                                  rp.layout.combination_count, w.as_ptr(), found_buf.as_ptr(), found_buf.len(), out.as_mut_ptr())
        })?;
        let payloads = out
            .chunks_exact(OMR_PAYLOAD_LEN)
            .map(|c| {
                let mut p = [0u16; OMR_PAYLOAD_LEN];
                p.copy_from_slice(c);
                p
            })
            .collect();
        Ok((found_buf, payloads))
    }
}

/// Library identification, e.g. "omr_gpu 0.1 gfx950".
pub fn version() -> String {
    unsafe { CStr::from_ptr(omr_version()) }.to_string_lossy().into_owned()
}
