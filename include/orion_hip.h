/*
 * orion_hip.h -- C-ABI of liborion_hip.so, the MI355X (gfx950) RNS-CKKS
 * backend for Orion.
 *
 * Part 1 is the drop-in boundary: exactly the symbol set Orion's Python layer
 * binds for its Lattigo backend (/root/reference/orion/backend/lattigo/
 * bindings.py:141-746, cgo exports in orion/backend/lattigo/<file>.go), with the
 * same argument meaning and int-handle semantics (lowest-free-id reuse,
 * minheap.go:46-64; *New ops allocate, in-place ops return their input id).
 * Each entry cites the Go export it replaces.  Plus the two symbols the fork's
 * Python layer calls that only its HEonGPU binding defines
 * (GenerateConsolidatedRotationKeys, lt_evaluator.py:77; CloneCiphertext,
 * tensors.py:229).
 *
 * Error behaviour: Lattigo panics (aborts the process).  This library never
 * aborts: handle-returning calls return -1, void calls record the error, and
 * OrionHipLastError() returns the message (the Python binding raises
 * RuntimeError).  Scalars and diagonals cross the ABI as 32-bit float, scales
 * as unsigned long, exactly like the Lattigo binding.
 *
 * Part 2 (OrionHip* and *Batch symbols) is new: batch ciphertexts (one handle
 * = B independent images, one kernel launch per op for the whole batch),
 * host/device import/export for parity tests and the RCCL key broadcast,
 * stream control and kernel timing.
 *
 * Every call is asynchronous on the library stream unless it returns data to
 * the host (Decode, Export*, Get*Scale never need to sync; Decode/Export do).
 */
#ifndef ORION_HIP_H
#define ORION_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { int *Data; unsigned long Length; } ArrayResultInt;          /* bindings.py:749-751 */
typedef struct { float *Data; unsigned long Length; } ArrayResultFloat;      /* bindings.py:753-754 */
typedef struct { double *Data; unsigned long Length; } ArrayResultDouble;    /* bindings.py:756-757 */
typedef struct { unsigned long *Data; unsigned long Length; } ArrayResultUInt64; /* bindings.py:759-760 */
typedef struct { char *Data; unsigned long Length; } ArrayResultByte;        /* bindings.py:762 */

/* ---------------- scheme (scheme.go:34-100, utils.go:93-95) ---------------- */
void NewScheme(int logN, int *logQ, int lenQ, int *logP, int lenP, int logScale, int h,
               char *ringType, char *keysPath, char *ioMode);                 /* scheme.go:35 */
void DeleteScheme(void);                                                   /* scheme.go:89 */
void FreeCArray(void *ptr);                                                /* utils.go:93 */

/* ---------------- tensors (tensors.go:36-123) ---------------- */
void DeletePlaintext(int id);                                              /* tensors.go:35 */
void DeleteCiphertext(int id);                                             /* tensors.go:40 */
unsigned long GetPlaintextScale(int id);                                   /* tensors.go:45 */
unsigned long GetCiphertextScale(int id);                                  /* tensors.go:53 */
void SetPlaintextScale(int id, unsigned long scale);                       /* tensors.go:61 */
void SetCiphertextScale(int id, unsigned long scale);                      /* tensors.go:67 */
int GetPlaintextLevel(int id);                                             /* tensors.go:73 */
int GetCiphertextLevel(int id);                                            /* tensors.go:79 */
int GetPlaintextSlots(int id);                                             /* tensors.go:85 */
int GetCiphertextSlots(int id);                                            /* tensors.go:92 */
int GetCiphertextDegree(int id);                                           /* tensors.go:99 */
ArrayResultUInt64 GetModuliChain(void);                                    /* tensors.go:105 */
ArrayResultInt GetLivePlaintexts(void);                                    /* tensors.go:112 */
ArrayResultInt GetLiveCiphertexts(void);                                   /* tensors.go:119 */
int CloneCiphertext(int id);                                               /* fork: tensors.py:229 */

/* ---------------- key generator (keygenerator.go:13-58) ---------------- */
void NewKeyGenerator(void);                                                /* keygenerator.go:13 */
void GenerateSecretKey(void);                                              /* keygenerator.go:18 */
void GeneratePublicKey(void);                                              /* keygenerator.go:23 */
void GenerateRelinearizationKey(void);                                     /* keygenerator.go:28 */
void GenerateEvaluationKeys(void);                                         /* keygenerator.go:33 */
/* Serialize / Load calls use Lattigo v6's MarshalBinary layouts (orion_amd/csrc/wire.h):
 * rlwe.SecretKey, rlwe.GaloisKey and ringqp.Poly, coefficients in Montgomery form */
ArrayResultByte SerializeSecretKey(void);                                  /* keygenerator.go:38 */
void LoadSecretKey(char *data, unsigned long len);                         /* keygenerator.go:49 */

/* ---------------- encoder / encryptor (encoder.go, encryptor.go) ---------------- */
void NewEncoder(void);                                                     /* encoder.go:11 */
int Encode(float *values, int lenValues, int level, unsigned long scale);  /* encoder.go:16 */
ArrayResultFloat Decode(int ptId);                                         /* encoder.go:33 */
void NewEncryptor(void);                                                   /* encryptor.go:10 */
void NewDecryptor(void);                                                   /* encryptor.go:15 */
int Encrypt(int ptId);                                                     /* encryptor.go:20 */
int Decrypt(int ctId);                                                     /* encryptor.go:30 */

/* ---------------- evaluator (evaluator.go:13-317) ---------------- */
void NewEvaluator(void);                                                   /* evaluator.go:14 */
void AddRotationKey(int rotation);                                         /* evaluator.go:34 */
int Negate(int ct);                                                        /* evaluator.go:49 */
int Rotate(int ct, int amount);                                            /* evaluator.go:61 */
int RotateNew(int ct, int amount);                                         /* evaluator.go:70 */
int Rescale(int ct);                                                       /* evaluator.go:84 */
int RescaleNew(int ct);                                                    /* evaluator.go:92 */
int AddScalar(int ct, float scalar);                                       /* evaluator.go:102 */
int AddScalarNew(int ct, float scalar);                                    /* evaluator.go:110 */
int SubScalar(int ct, float scalar);                                       /* evaluator.go:122 */
int SubScalarNew(int ct, float scalar);                                    /* evaluator.go:130 */
int MulScalarInt(int ct, int scalar);                                      /* evaluator.go:142 */
int MulScalarIntNew(int ct, int scalar);                                   /* evaluator.go:150 */
int MulScalarFloat(int ct, float scalar);                                  /* evaluator.go:162 */
int MulScalarFloatNew(int ct, float scalar);                               /* evaluator.go:170 */
int AddPlaintext(int ct, int pt);                                          /* evaluator.go:182 */
int AddPlaintextNew(int ct, int pt);                                       /* evaluator.go:191 */
int SubPlaintext(int ct, int pt);                                          /* evaluator.go:205 */
int SubPlaintextNew(int ct, int pt);                                       /* evaluator.go:214 */
int MulPlaintext(int ct, int pt);                                          /* evaluator.go:228 */
int MulPlaintextNew(int ct, int pt);                                       /* evaluator.go:237 */
int AddCiphertext(int ct0, int ct1);                                       /* evaluator.go:251 */
int AddCiphertextNew(int ct0, int ct1);                                    /* evaluator.go:260 */
int SubCiphertext(int ct0, int ct1);                                       /* evaluator.go:274 */
int SubCiphertextNew(int ct0, int ct1);                                    /* evaluator.go:283 */
int MulRelinCiphertext(int ct0, int ct1);                                  /* evaluator.go:297 */
int MulRelinCiphertextNew(int ct0, int ct1);                               /* evaluator.go:306 */

/* ---------------- linear transforms (lineartransform.go:26-211) ---------------- */
void NewLinearTransformEvaluator(void);                                    /* lineartransform.go:31 */
int GenerateLinearTransform(int *diagIdx, int nIdx, float *diagData, int nData, int level,
                            float bsgsRatio, char *ioMode);                /* lineartransform.go:37 */
int EvaluateLinearTransform(int transformId, int ctId);                    /* lineartransform.go:96 */
void DeleteLinearTransform(int id);                                        /* lineartransform.go:26 */
ArrayResultInt GetLinearTransformRotationKeys(int transformId);            /* lineartransform.go:116 */
void GenerateLinearTransformRotationKey(int galEl);                        /* lineartransform.go:125 */
void GenerateConsolidatedRotationKeys(int *galEls, int n);                 /* fork: lt_evaluator.py:77 */
ArrayResultByte GenerateAndSerializeRotationKey(int galEl);                /* lineartransform.go:131 */
/* LoadRotationKey keeps a key in HBM only over the limbs and digits of the
 * highest level at which the linear transforms existing at load time use it
 * (a key with no such transform is kept whole); the cut keeps ResNet-20's
 * ~120 keys in a few GB of HBM instead of ~150 GB.  The whole key stays in
 * host memory, as Lattigo keeps it (lineartransform.go:143-159): a later use
 * above the cut level uploads it whole, the loaded key itself. */
void LoadRotationKey(char *data, unsigned long len, unsigned long galEl);  /* lineartransform.go:143 */
ArrayResultByte SerializeDiagonal(int transformId, int diagIdx);           /* lineartransform.go:162 */
void LoadPlaintextDiagonal(char *data, unsigned long len, int transformId,
                           unsigned long diagIdx);                         /* lineartransform.go:180 */
void RemovePlaintextDiagonals(int transformId);                            /* lineartransform.go:196 */
void RemoveRotationKeys(void);                                             /* lineartransform.go:204 */

/* ---------------- polynomial evaluator / bootstrapping ----------------
 * Implemented on the GPU: Lattigo's polynomial evaluator
 * (power basis + Paterson-Stockmeyer, level and target-scale contract) and
 * one bootstrapper per slot count under bootstrapping parameters of its own
 * (residual Q + 15 circuit primes, P primes of the bit sizes logPs), with
 * Orion's post-scale 2^(LogMaxSlots - LogSlots).  */
void NewPolynomialEvaluator(void);                                         /* polyeval.go:33 */
int GenerateMonomial(float *coeffs, int n);                                /* polyeval.go:38 */
int GenerateChebyshev(float *coeffs, int n);                               /* polyeval.go:50 */
int EvaluatePolynomial(int ct, int poly, unsigned long outScale);          /* polyeval.go:63 */
ArrayResultDouble GenerateMinimaxSignCoeffs(int *degrees, int n, int prec, int logalpha,
                                            int logerr, int debug);        /* polyeval.go:91 */
void NewBootstrapper(int *logPs, int n, int slots);                        /* bootstrapper.go:19 */
int Bootstrap(int ct, int slots);                                          /* bootstrapper.go:61 */
void DeleteBootstrappers(void);                                            /* bootstrapper.go:91 */

/* ---- the fork's Python layer beyond the Lattigo set ---- */
int ModDropCiphertext(int ct);     /* evaluator.py:30-41 (HEonGPU _ModDropCiphertext): drop the top modulus, in place */
int GetPolyDepth(int poly);        /* poly_evaluator.py:58-59: levels EvaluatePolynomial consumes */

/* ================= Part 2: MI355X extensions ================= */
const char *OrionHipLastError(void);
void OrionHipClearError(void);
int OrionHipSetDevice(int device);
void OrionHipSetSeed(unsigned long seed);                /* keygen / encryption PRNG seed */
void OrionHipSetStream(void *hipStream);                  /* NULL = library-owned stream */
void *OrionHipGetStream(void);
/* Pipelines (thread-affine contexts).  The reference's scheme is a process
 * singleton (orion/core/orion.py:323; Lattigo's global state, scheme.go:32);
 * here each thread acts on one context of the scheme.  A pipeline is a context
 * on the scheme's chain that shares the scheme's keys and reads its compiled
 * objects (plaintexts, linear transforms, polynomials, bootstrappers), with
 * its own HIP stream, buffer pool and handle range; calls acting on different
 * contexts run concurrently (each holds only its own context's lock), so
 * several threads each running the frontend's `net(ct)` overlap on the GPU.
 *
 * OrionHipThreadPipelines(n): n > 1 gives every thread other than the one that
 * called NewScheme a pipeline of its own at its first call (up to n contexts,
 * then shared round-robin); n <= 1 (default; or ORION_THREAD_PIPELINES=n in
 * the environment) leaves every thread on the scheme's context.  Returns the
 * previous setting.  OrionHipCurrentPipeline: the calling thread's context
 * index (0 = the scheme's).  OrionHipPeerCreate makes a pipeline and returns
 * its index without binding a thread; OrionHipPeerSelect(id) binds the
 * calling thread to context id.  Handles are unique across contexts: a call
 * naming another context's object orders its stream after that object's
 * producer; deletes and metadata calls go to the handle's own context; an
 * in-place op on another context's ciphertext is refused.  DeleteScheme
 * removes every pipeline. */
int OrionHipThreadPipelines(int n);
int OrionHipCurrentPipeline(void);
int OrionHipPeerCreate(void);
int OrionHipPeerSelect(int id);
int OrionHipPeerCount(void);
/* The calling thread's context's stream waits (on the GPU) for the work
 * enqueued so far on context `peer`'s stream (an event recorded there).
 * A frontend uses it to start one pipeline behind another.  0 or -1. */
int OrionHipStreamWaitPeer(int peer);

/* Device-memory pools of the process (one per context: the scheme's, its
 * pipelines', the bootstrappers'): out[0] bytes held (handed out + cached),
 * out[1] their peak, out[2] hipMalloc calls, out[3] failed allocations that
 * forced every pool to release its cache (then one retry), out[4] bytes
 * cached; returns the number of fields. */
int OrionHipPoolStats(double* out, int n);
/* A cap on the bytes all pools hold together (0: none; also
 * ORION_POOL_CAP_BYTES): an allocation past it takes the failed-hipMalloc
 * path -- release every cache, retry once, else fail the call with "device
 * memory exhausted".  Returns the previous cap. */
double OrionHipPoolCap(double bytes);
int OrionHipSynchronize(void); /* drains every context's stream */
/* hipGraph capture of an op stream issued through this ABI: every call between
 * Begin and End is recorded into one graph (returned id), which Launch replays
 * on the library stream with one launch, into the same buffers (the pool pins
 * them until Destroy).  The captured calls must not need a synchronisation:
 * run the stream once before capturing it (keys, tables, LT plans). */
/* ct += Rotate(ct, amount), in place: the same result as RotateNew(ct, amount)
 * followed by AddCiphertext(ct, <that rotation>) (evaluator.go:70 + :251), the
 * addition done in the key switch's final store.  The replay uses it when a
 * rotation's only consumer is that addition (LoLA's rotate-and-sum). */
int OrionHipRotateAdd(int ct, int amount);
int OrionHipGraphBegin(void);
int OrionHipGraphEnd(void);                               /* graph id, or -1 */
int OrionHipGraphLaunch(int graph);
void OrionHipGraphDestroy(int graph);
int OrionHipLogN(void);                                   /* log2 of the ring degree N (coefficients per limb) */
int OrionHipNumQ(void);
int OrionHipNumP(void);
unsigned long OrionHipModulus(int idx);                   /* QP index space */
/* the bootstrapping chain of the circuit for `slots` (NewBootstrapper):
 * Q primes (residual + circuit), then P primes; -1 / 0 when there is none */
int OrionHipBootstrapNumQ(int slots);
int OrionHipBootstrapNumP(int slots);
unsigned long OrionHipBootstrapModulus(int slots, int idx);
/* parity access to the shared inputs of the circuit for `slots` (keys,
 * diagonals, constants), so that the CPU oracle can restate the circuit on
 * the same inputs (tests only).  Returns the element count written, or needed
 * when out is NULL; -1 on error.  Items (element type):
 *   PARAMS (long double): F, gap, K, r, degree, slots, s_y, top, L, K_P,
 *          #trace rotations, #transforms, #cosine coefficients, t0 (EvalMod
 *          polynomial target scale)
 *   COS (long double): EvalMod's Chebyshev coefficients, lowest first
 *   TRACE (unsigned long): Galois elements of the trace
 *   RLK / GALOIS (arg = galEl) (unsigned long): key in the full-chain layout
 *          [dnum][2][L+K][N] of the bootstrapping chain
 *   GALOIS_KEYS (unsigned long): every Galois element with a key
 *   LT_INFO (arg = transform 0..5, CoeffsToSlots then SlotsToCoeffs) (long):
 *          level, N1, #diagonals, diagonal indices
 *   LT_DIAG (arg = transform << 32 | k) (unsigned long): k-th diagonal,
 *          [level+1+K_P][N] NTT domain
 *   MONO_I (unsigned long): X^(N/2) over the Q limbs, NTT domain (full slots)
 *   D2S / S2D (unsigned long): the ephemeral-secret keys EvkDenseToSparse
 *          (made for level 0) and EvkSparseToDense, full-chain layout
 * The CPU oracle takes only the keys (RLK, GALOIS, D2S, S2D) and derives the
 * constants, diagonals and prime chain itself; the other items let the tests
 * compare the two derivations. */
enum { ORION_BTX_PARAMS = 0, ORION_BTX_COS, ORION_BTX_TRACE, ORION_BTX_RLK, ORION_BTX_GALOIS_KEYS,
       ORION_BTX_GALOIS, ORION_BTX_LT_INFO, ORION_BTX_LT_DIAG, ORION_BTX_MONO_I, ORION_BTX_D2S, ORION_BTX_S2D };
long OrionHipBootstrapExport(int slots, int what, long arg, void *out, unsigned long n);

/* batch ciphertexts: one handle holds B images; ops act on the whole batch */
int EncodeBatch(float *values, int lenPerImage, int batch, int level, unsigned long scale);
int GetCiphertextBatch(int ct);
int GetPlaintextBatch(int pt);
double GetCiphertextScaleF(int ct);                       /* exact-ish scale (long double -> double) */

/* GPU encoder with device-resident slots (e.g. a torch tensor's data_ptr):
 * dvalues [batch][lenPerImage] float32; DecodeDevice writes the real parts of
 * all slots, [batch][N/2] float64, to device memory (asynchronous);
 * DecodeF64 returns them to the host as float64 (Decode casts to float32) */
int EncodeBatchDevice(const float *dvalues, int lenPerImage, int batch, int level, double scale);
int DecodeDevice(int pt, double *dout);
int DecodeF64(int pt, double *out, unsigned long n);
/* encryption randomness: ChaCha20 stream keyed from the seed (OrionHipSetSeed
 * / NewScheme), nonce = (encryption index, image, component); the index counts
 * Encrypt calls since the last seeding */
unsigned int OrionHipEncryptionIndex(void);

/* host import/export, canonical host layout [batch][comp][limb][N] (NTT) */
int ImportCiphertext(const unsigned long *data, int batch, int level, double scale);
int ExportCiphertext(int ct, unsigned long *out, unsigned long n);
int ImportPlaintext(const unsigned long *data, int batch, int level, double scale);
int ExportPlaintext(int pt, unsigned long *out, unsigned long n);
/* the same canonical layout in device memory (e.g. a torch.uint64/int64 tensor
 * on the library's GPU): no host round trip, asynchronous on the library stream.
 * Ordering is the caller's: the library stream (OrionHipGetStream) must wait
 * for the work that writes dptr before an import (and the buffer must not be
 * freed or reused until the copy has run), and a consumer of an export must
 * wait for the library stream.  orion_amd/backend.py does this with stream
 * waits and record_stream; the same holds for EncodeBatchDevice's dvalues and
 * DecodeDevice's dout.  Residues must be fully reduced in [0, q_l): kernels
 * assume it and the import does not check. */
int ImportCiphertextDevice(const unsigned long *dptr, int batch, int level, double scale);
int ExportCiphertextDevice(int ct, unsigned long *dptr, unsigned long n);
int ExportSecretKey(unsigned long *out, unsigned long n);                  /* [L+K][N]           */
int ExportPublicKey(unsigned long *out, unsigned long n);                  /* [2][L+K][N]        */
int ExportRelinKey(unsigned long *out, unsigned long n);                   /* [dnum][2][L+K][N]  */
int ExportGaloisKey(unsigned long galEl, unsigned long *out, unsigned long n);  /* full layout, zero past its level */
/* Galois keys are made for the highest level they are needed at (a linear
 * transform's level for its rotations, L-1 otherwise); a key made for level l
 * holds ceil((l+1)/K) digits over l+1+K limbs */
int GetGaloisKeyLevel(unsigned long galEl);
int ExportLinearTransformDiagonal(int lt, int diagIdx, unsigned long *out, unsigned long n); /* [lvl+1+K][N] */
int GetLinearTransformN1(int lt);
unsigned long GaloisElement(int rotation);

/* key bundle (public + evaluation keys [+ secret]) as one device buffer, for
 * RCCL broadcast over xGMI; dptr is device memory owned by the caller */
unsigned long KeyBundleBytes(int withSecret);
int ExportKeyBundle(void *dptr, int withSecret);
int ImportKeyBundle(const void *dptr, unsigned long bytes);

/* kernel timing with HIP events on the library stream; enable: 0 = off,
 * 1 = every category, otherwise a bit mask of categories (bit 0 ntt_fwd,
 * 1 ntt_inv, 2 elementwise, 3 basis_ext, 4 ks_mac, 5 automorph, 6 tensor,
 * 7 rescale_prep, 8 lt_bsgs, 9 lt_giant) */
void OrionHipProfile(int enable);
/* fills up to max entries: name (32 chars each), launches, total ms, algorithmic
 * bytes (NTT: 16 N per limb-transform + 8 N per epilogue operand or addend read,
 * the "fused" model; the automorphism scatter index is not counted) */
int OrionHipProfileRead(char *names, long *launches, double *ms, double *bytes, int max);
/* the same categories priced strictly as SURVEY §8d does: 16 N per NTT
 * limb-transform, whatever the prologue and epilogue read (other categories:
 * equal to their algorithmic bytes) */
int OrionHipProfileReadStrict(double *strict, int max);
void OrionHipProfileReset(void);
/* union timing across contexts (peer pipelines): ProfileClock records the
 * reference and drops the collected intervals; ProfileUnion returns the
 * wall-clock length (ms) of the union of the intervals of every context's
 * profiled launches of the categories in `mask` since then */
void OrionHipProfileClock(void);
/* a marker line "# tag" in the ORION_NTT_LOG call log (no-op without it) */
void OrionHipLogMark(const char *tag);
double OrionHipProfileUnion(unsigned mask);

/* raw kernel entry for the roofline microbenchmark and parity tests:
 * in-place NTT/INTT of `nlimb` limbs x `batch` images at device pointer
 * (layout [limb][batch][N]), limb l under QP modulus index mods[l];
 * inverse bit 0: INTT; bit 1: out of place, into the nlimb x batch limbs
 * that follow the input */
int OrionHipNTT(unsigned long *dptr, int nlimb, int batch, const int *mods, int inverse);

#ifdef __cplusplus
}
#endif
#endif
