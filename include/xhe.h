/* xhe — MI355X (gfx950) Paillier hot path, C ABI.
 *
 * Drop-in boundary for XFL's python/common/crypto/paillier (reference paths
 * below are relative to /root/reference/python). Every entry point takes plain
 * pointers and sizes; "_dev" pointers are device (HBM) buffers owned by the
 * caller, "_host" entry points take host buffers and do the H2D/D2H copies.
 * Big integers are little-endian arrays of 32-bit words:
 *   n: nw = key_bits/32 words, ciphertexts (mod n^2): n2w = 2*nw words,
 *   randomness a (DJN) / r (non-DJN): rand_words words per element.
 * Return value: 0 on success, negative XHE_E* on failure; xhe_last_error()
 * gives the thread-local message. A key handle is immutable after creation
 * and may be shared between threads; calls on distinct streams are reentrant.
 */
#ifndef XHE_H
#define XHE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XHE_OK 0
#define XHE_EINVAL -1     /* bad argument (TypeError/ValueError side)          */
#define XHE_EOVERFLOW -2  /* value out of the encodable/decodable range        */
#define XHE_EHIP -3       /* HIP runtime error                                  */
#define XHE_ENOINV -4     /* no modular inverse (ZeroDivisionError)             */
#define XHE_ENOTSUP -5    /* mode not built for this key size                   */

typedef struct xhe_key xhe_key;

/* Key material -> device key handle with all per-key precomputes
 * (PaillierContext.init, context.py:28-71) and, for a DJN private key, the
 * fixed-base tables of h_pow_n mod p^2 / q^2 (2^win rows per window).
 * p_words/q_words NULL => public key (n only). h_pow_n_words NULL => DJN off.
 * p, q: nw/2 words each; h_pow_n: n2w words. win_bits: the window w in
 * [2, 24], 0 = default (16, or $XHE_WIN_BITS); tables take ceil(rand_bits/w)
 * windows of 2^w packed rows (K/32 words) per prime. With XHE_WIN_SPLIT or'ed
 * in (w <= 23): floor(rand_bits/w) windows, the first rand_bits mod w of them
 * w+1 bits wide (one table product fewer for ~1.25x the rows). 2048-bit key
 * (rand_bits 1024), per prime: w 16: 1.07 GB, 64 products; 20: 14 GB, 52;
 * 22: 50.5 GB, 47; 23: 96.6 GB, 45; 23 split: 120.3 GB, 44.
 * key_bits: 2048, 3072, 4096 or 8192 (else XHE_ENOTSUP). */
#define XHE_WIN_SPLIT 0x100
int xhe_key_create(int device, int key_bits, const uint32_t* n_words, const uint32_t* p_words,
                   const uint32_t* q_words, const uint32_t* h_pow_n_words, int win_bits, xhe_key** out);
void xhe_key_destroy(xhe_key* key);
/* nw, n2w, rand_words (32-bit words per randomness draw), rand_bits
 * (DJN: bitlen(n)//2 = log2 djn_exp_bound; non-DJN: bitlen(n)), flags bit0
 * private, bit1 djn. */
int xhe_key_info(const xhe_key* key, int* key_bits, int* nw, int* n2w, int* rand_words, int* rand_bits, int* flags);

/* PaillierEncoder.cal_exponent + encode_single over float64 (encoder.py:29-54,
 * paillier.py:279-282). precision < 0 => None (frexp exponent), else
 * e = -ceil(log2(10)*precision). has_max => e = min(e, max_exponent).
 * Per element: m (nw words), exponent, status (0, 1 = OverflowError, 2 = ValueError). */
int xhe_encode_f64(const xhe_key* key, const double* x_dev, int64_t count, int precision, int has_max,
                   int max_exponent, uint32_t* m_dev, int32_t* exp_dev, int32_t* status_dev, void* stream);

/* Obfuscation randomness from a ChaCha20 stream keyed by seed32 (32 bytes) and
 * nonce: DJN a in [1, djn_exp_bound) (paillier.py:195,211) or non-DJN r in
 * [1, n) (paillier.py:215,229). Replaces secrets.SystemRandom().randrange. */
int xhe_rand(const xhe_key* key, const uint8_t* seed32, uint64_t nonce, int64_t count, uint32_t* rand_dev,
             int32_t* status_dev, void* stream);

/* Paillier._encrypt_single + PaillierCiphertext.obfuscate (paillier.py:273-287,
 * 189-232): ct = (1 + n*m) * X mod n^2 with X from rand (NULL = no obfuscation). */
int xhe_encrypt(const xhe_key* key, const uint32_t* m_dev, const uint32_t* rand_dev, int64_t count,
                uint32_t* ct_dev, void* stream);

/* Paillier._decrypt_single arithmetic (paillier.py:341-366): ct -> encoded m. */
int xhe_decrypt(const xhe_key* key, const uint32_t* ct_dev, int64_t count, uint32_t* m_dev, void* stream);

/* PaillierEncoder.decode_single + astype(np.float32) (encoder.py:56-64,
 * paillier.py:396-398): f64 = value before the float32 cast, f32 = result;
 * status 1 = OverflowError (decode range), 3 = OverflowError (mpz->float). */
int xhe_decode(const xhe_key* key, const uint32_t* m_dev, const int32_t* exp_dev, int64_t count, double* f64_dev,
               float* f32_dev, int32_t* status_dev, void* stream);

/* Ciphertext addition PaillierCiphertext._add_encrypted (paillier.py:106-123,
 * 79-86, 153-154): out = a' * b' mod n^2 where the operand with the larger
 * exponent is first raised to 2^(e - min(ea, eb)); eout = min(ea, eb).
 * ea/eb may be NULL (all 0). dmax >= max |ea - eb| bounds the squarings.
 * As in the reference, a gap d with 2^d >= min_value_for_negative (d >=
 * ~bitlen(n) - 1) takes _raw_mul's negative branch: that operand is raised to
 * 2^d - n instead (paillier.py:79-86, 173-187; same plaintext, other bits). */
int xhe_mulmod(const xhe_key* key, const uint32_t* a_dev, const int32_t* ea_dev, const uint32_t* b_dev,
               const int32_t* eb_dev, int64_t count, int dmax, uint32_t* out_dev, int32_t* eout_dev, void* stream);
/* PaillierCiphertext._raw_mul positive branch (paillier.py:156-187):
 * out = c^k mod n^2, k per element (kw words, k < 2^kbits). */
int xhe_powmod(const xhe_key* key, const uint32_t* c_dev, const uint32_t* k_dev, int kw, int kbits, int64_t count,
               uint32_t* out_dev, void* stream);
/* utils.invert over n^2 (utils.py:71-76) for a batch: out = c^-1 mod n^2
 * (product-tree batch inversion). XHE_ENOINV when some c has no inverse. */
int xhe_invert(const xhe_key* key, const uint32_t* c_dev, int64_t count, uint32_t* out_dev, void* stream);

/* Homomorphic sum per segment (np.sum / pandas groupby('bin').sum() over
 * ciphertexts, decision_tree_trainer.py:151-160, xgb_actor.py:340-345,447-456):
 * out[s] = prod_{i in [seg_begin[s], seg_begin[s+1])} c_i^(2^d_i) mod n^2,
 * d_i = e_i - (min exponent of the segment) (NULL = all 0), dmax >= max d_i.
 * seg_begin is a HOST array of nseg+1 offsets into the segment-ordered input;
 * an empty segment yields 1 (the encryption of 0 without obfuscation).
 * This is the order-free fold: equal to any order of the reference's
 * pairwise adds while every gap is below the negative-branch threshold
 * (see xhe_mulmod); past it the reference's bits depend on the addition tree,
 * and the caller pre-aligns those elements (xfl_amd/paillier/ops.py
 * segment_sums_words). */
int xhe_segprod(const xhe_key* key, const uint32_t* c_dev, const int32_t* d_dev, int dmax, int64_t count,
                const int64_t* seg_begin, int64_t nseg, uint32_t* out_dev, void* stream);

/* Encrypted matrix-vector product as a multi-exponentiation: the object-dtype
 * np.matmul(enc[B], X[B, D]) of logistic_regression/trainer.py:166 (and
 * linear_regression/trainer.py:207, poisson_regression/trainer.py:267,
 * pearson/trainer.py:120-123), i.e. per column j the fold of
 * PaillierCiphertext.__mul__ + __add__ (paillier.py:106-187), is
 *   out[j] = prod_{t < nterms} bases[idx[j*nterms + t]]^k[j*nterms + t] mod n^2
 * with the caller folding signs (base = c or c^-1, xhe_invert) and exponent
 * alignment (k << (e - e_min)) into idx/k. k: kw words per term, < 2^kbits.
 * Straus windows of win_bits (0 = chosen to minimise products) with per-base
 * tables shared by all columns. */
int xhe_multiexp(const xhe_key* key, const uint32_t* bases_dev, int64_t nbases, const int32_t* idx_dev,
                 const uint32_t* k_dev, int kw, int kbits, int64_t ncols, int64_t nterms, int win_bits,
                 uint32_t* out_dev, void* stream);

/* Row moves of device ciphertext arrays (words per row), the element
 * selection and assignment of the flat arrays the drop-in returns (fancy
 * indexing and views of the reference's np.ndarray[object] results,
 * paillier.py:289-339): gather dst[i] = src[idx[i]] and scatter dst[idx[i]] =
 * src[i], idx a DEVICE int64 array of count rows (every idx < the row count of
 * the indexed array; scatter indices distinct). On the device this library
 * already holds, so no other runtime's kernels are loaded on first use. */
int xhe_gather_rows(const uint32_t* src_dev, const int64_t* idx_dev, int64_t count, int words, uint32_t* dst_dev,
                    void* stream);
int xhe_scatter_rows(const uint32_t* src_dev, const int64_t* idx_dev, int64_t count, int words, uint32_t* dst_dev,
                     void* stream);
/* bits_dev[i] = bit length of row i of words_dev (count x n2w little-endian
 * words, n2w <= 1023): the per-element input of xhe_wire_layout, so the
 * serialize payload is sized before the ciphertexts are downloaded. */
int xhe_row_bits(const uint32_t* words_dev, int64_t count, int n2w, int16_t* bits_dev, void* stream);
/* Host only (no device): the constant blocks k_dec_rns reads for the prime P
 * (p_words: pw words) - the bases' block (shared_out: XHE_RNS_SHARED_WORDS)
 * and P's block (prime_out: XHE_RNS_PRIME_WORDS); for tests against
 * tools/rns_model.py. */
#define XHE_RNS_SHARED_WORDS 19784
#define XHE_RNS_PRIME_WORDS 2088
int xhe_rns_constants(const uint32_t* p_words, int pw, uint32_t* shared_out, uint32_t* prime_out);

/* Host-buffer variants (H2D -> kernels -> D2H on an internal stream). */
int xhe_multiexp_host(const xhe_key* key, const uint32_t* bases, int64_t nbases, const int32_t* idx, const uint32_t* k,
                      int kw, int kbits, int64_t ncols, int64_t nterms, int win_bits, uint32_t* out);
int xhe_segprod_host(const xhe_key* key, const uint32_t* c, const int32_t* d, int dmax, int64_t count,
                     const int64_t* seg_begin, int64_t nseg, uint32_t* out);
int xhe_mulmod_host(const xhe_key* key, const uint32_t* a, const int32_t* ea, const uint32_t* b, const int32_t* eb,
                    int64_t count, int dmax, uint32_t* out, int32_t* eout);
/* c^k (or (c^-1)^k when invert_first: the negative-scalar branch). */
int xhe_powmod_host(const xhe_key* key, const uint32_t* c, const uint32_t* k, int kw, int kbits, int64_t count,
                    int invert_first, uint32_t* out);
/* Paillier.encrypt over a float64 array (paillier.py:289-339): encode + (device
 * ChaCha20 randomness when obfuscate) + encrypt; ct, exponent and encode
 * status per element. */
int xhe_encrypt_f64_host(const xhe_key* key, const double* x, int64_t count, int precision, int has_max,
                         int max_exponent, int obfuscate, const uint8_t* seed32, uint64_t nonce, uint32_t* ct,
                         int32_t* exps, int32_t* status);
/* Paillier.encrypt of already-encoded integers m (nw words each). */
int xhe_encrypt_words_host(const xhe_key* key, const uint32_t* m, int64_t count, int obfuscate,
                           const uint8_t* seed32, uint64_t nonce, uint32_t* ct);
/* Paillier.decrypt(dtype='float') (paillier.py:370-398): decrypt + decode;
 * m_out (nullable) receives the encoded integers. */
int xhe_decrypt_decode_host(const xhe_key* key, const uint32_t* ct, const int32_t* exps, int64_t count, double* f64,
                            float* f32, int32_t* status, uint32_t* m_out);
int xhe_encrypt_host(const xhe_key* key, const uint32_t* m, const uint32_t* rand, int64_t count, uint32_t* ct);
int xhe_decrypt_host(const xhe_key* key, const uint32_t* ct, int64_t count, uint32_t* m);

/* Wire codec (host only, no device needed): the byte format of
 * Paillier.serialize / Paillier.ciphertext_from (paillier.py:244-271,
 * compression=False; zstd framing stays in the caller) — a pickle of an
 * np.ndarray(dtype=object) of RawCiphertext(value, exp) — to and from flat
 * buffers (ct: count x n2w little-endian words). encode: XHE_EOVERFLOW with
 * *out_len = bytes needed when cap is too small (out may be NULL). decode:
 * accepts CPython's pickles of that object graph at protocols 2-5, including
 * the reference's gmpy2 mpz values; XHE_EOVERFLOW with *count set when
 * cap_count is too small; XHE_EINVAL on anything else. */
int xhe_wire_encode(const uint32_t* ct, const int32_t* exps, int64_t count, int n2w, const int64_t* shape, int ndim,
                    uint8_t* out, int64_t cap, int64_t* out_len);
int xhe_wire_decode(const uint8_t* data, int64_t len, int n2w, uint32_t* ct, int32_t* exps, int64_t cap_count,
                    int64_t* count, int64_t* shape, int* ndim);
/* xhe_wire_encode written straight into its final bytes: framed == 0 gives
 * the same pickle; framed != 0 gives xhe_zstd_raw_frame(pickle) - what
 * Paillier.serialize(compression=True) sends (paillier.py:244-258) - without
 * the intermediate pickle buffer. *out_len = the bytes needed; XHE_EOVERFLOW
 * when cap is smaller (out may be NULL). */
int xhe_wire_encode_frame(const uint32_t* ct, const int32_t* exps, int64_t count, int n2w, const int64_t* shape,
                          int ndim, int framed, uint8_t* out, int64_t cap, int64_t* out_len);
/* The same bytes in two steps, for words that arrive chunk by chunk (the
 * serialize pipeline overlaps the D2H copy of one chunk with the encoding of
 * the previous one). layout: elem_off[0..count] = each element's pickle
 * offset (elem_off[count]: the footer), from the bit lengths (xhe_row_bits);
 * *out_len = the payload size; with out (cap >= it) also the header, the
 * footer and, framed, the zstd frame and block headers. rows: elements
 * lo..hi-1 (rows[0] = element lo) at those offsets; XHE_EINVAL when a row's
 * bit length differs from the layout's. */
int xhe_wire_layout(const int16_t* bits, const int32_t* exps, int64_t count, int n2w, const int64_t* shape, int ndim,
                    int framed, int64_t* elem_off, uint8_t* out, int64_t cap, int64_t* out_len);
int xhe_wire_rows(const uint32_t* rows, const int32_t* exps, int64_t lo, int64_t hi, int64_t count, int n2w,
                  const int64_t* elem_off, int framed, uint8_t* out, int64_t cap);
/* The layout range by range, for bit lengths that arrive chunk by chunk
 * too (a serialize that starts while the encryption runs): begin sets
 * elem_off[0] and *max_len = the payload size if every element had the
 * largest bit length n2w words allow (allocate that), and with out writes the
 * header; layout_part fills elem_off[lo+1..hi] from elem_off[lo] and the bit
 * lengths of elements lo..hi-1 (bits[0] = element lo); rows as above, for
 * ranges laid out so far; finish writes the footer and, framed, the zstd frame
 * and block headers, and sets *out_len = the payload's real size (the caller
 * cuts its buffer to it). The bytes equal xhe_wire_encode_frame's. */
int xhe_wire_begin(const int32_t* exps, int64_t count, int n2w, const int64_t* shape, int ndim, int framed,
                   int64_t* elem_off, int64_t* max_len, uint8_t* out, int64_t cap);
int xhe_wire_layout_part(const int16_t* bits, const int32_t* exps, int64_t lo, int64_t hi, int64_t count, int n2w,
                         int64_t* elem_off);
/* layout_part from the rows' own words (rows[0] = element lo) instead of
 * device-computed bit lengths. */
int xhe_wire_layout_part_rows(const uint32_t* rows, const int32_t* exps, int64_t lo, int64_t hi, int64_t count,
                              int n2w, int64_t* elem_off);
int xhe_wire_finish(int64_t count, const int64_t* elem_off, int framed, uint8_t* out, int64_t cap, int64_t* out_len);

/* A zstd frame (RFC 8878, one frame, content size in the header) holding
 * src[0..n) as raw blocks, written by several host threads: what
 * Paillier.serialize(compression=True) sends for large arrays
 * (paillier.py:244-258 zstd.compress). Ciphertext bytes are incompressible
 * (zstd level 3 keeps 98 % of a pickled ciphertext array), so the frame
 * costs a parallel copy instead of a single-threaded entropy search, and any
 * zstd decoder (the reference's zstd.decompress) reads it back. *out_len =
 * the frame's size (xhe_zstd_raw_frame_size(n)); XHE_EOVERFLOW when cap is
 * smaller (dst may be NULL). */
int64_t xhe_zstd_raw_frame_size(int64_t n);
int xhe_zstd_raw_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t* out_len);
/* Its inverse for frames made only of raw blocks, copied out in parallel
 * (ciphertext_from(compression=True), paillier.py:260-264): *out_len = the
 * content size; XHE_ENOTSUP for any other frame (the caller then uses
 * libzstd), XHE_EOVERFLOW when cap is too small. */
int xhe_zstd_raw_extract(const uint8_t* src, int64_t len, uint8_t* dst, int64_t cap, int64_t* out_len);

/* Touch every page of a fresh host buffer from several threads (host only),
 * so results copied in later do not take the first-touch faults on one
 * thread; the bytes become zero. Used for the hundreds-of-MB ciphertext
 * arrays of the drop-in (Paillier.encrypt's return, paillier.py:289-339). */
int xhe_host_prefault(void* p, int64_t nbytes);

/* Kernel timing: when enabled, the library brackets each launch of its
 * dominant kernels (k_djn_pow, k_dec_pow) with hipEvents on the launch stream.
 * xhe_profile(1) enables and clears, xhe_profile(0) disables and clears;
 * xhe_profile_read sums the recorded durations of `kernel` (NULL = all). */
int xhe_profile(int enable);
int xhe_profile_read(const char* kernel, double* total_ms, int64_t* launches);

int xhe_device_count(void);
int xhe_synchronize(void* stream);
const char* xhe_last_error(void);
const char* xhe_version(void);

#ifdef __cplusplus
}
#endif
#endif
