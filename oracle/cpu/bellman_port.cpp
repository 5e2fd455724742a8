// ORACLE / CPU BASELINE (test + bench infrastructure only; never linked into the
// product).  A C++ restatement of bellman's multicore Groth16 prover core, used
//   (a) as the "port" CPU baseline bench.py times on the GPU box's host cores;
//   (b) as an independent medium-size parity check (its proof bytes must equal
//       the device prover's on the same witness and Parameters).
// It keeps the reference's ALGORITHM and parallel structure, not just its result:
//   * multiexp.rs:159-281  window c = 3 if n < 32 else ceil(ln n); one task per
//     window (skip = 0, c, 2c, .. < 255), each scanning all n exponents with the
//     density/skip semantics; bucket[digit-1] mixed adds, summation by parts,
//     Horner combine over the windows.
//   * prover.rs:233-307    all 8 multiexps are in flight at once (Worker::compute),
//     their window tasks share one thread pool (rayon's).
//   * domain.rs:261-372    best_fft -> parallel_fft with P = 2^floor(log2 threads)
//     (size-P DFT shuffle, serial_fft of size n/P, transpose), serial_fft when
//     log_n <= log_threads; pointwise ops chunked over the threads.
//   * prover.rs:210-231    ifft/coset_fft x3, mul, sub, divide_by_z, icoset_fft.
// Field/curve arithmetic: 64-bit-limb Montgomery (the bls12_381 0.6 layout),
// Jacobian coordinates.  Build: oracle/cpu/Makefile -> oracle/cpu/libbellman_port.so
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

typedef unsigned __int128 u128;

// ===================================================================== fields
static const uint64_t P_[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                               0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
static const uint64_t PINV_ = 0x89f3fffcfffcfffdull;
static const uint64_t PR2_[6] = {0xf4df1f341c341746ull, 0x0a76e6a609d104f1ull, 0x8de5476c4c95b6d5ull,
                                 0x67eb88a9939d83c0ull, 0x9a793e85b519952dull, 0x11988fe592cae3aaull};
static const uint64_t PONE_[6] = {0x760900000002fffdull, 0xebf4000bc40c0002ull, 0x5f48985753c758baull,
                                  0x77ce585370525745ull, 0x5c071a97a256ec6dull, 0x15f65ec3fa80e493ull};
static const uint64_t Q_[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                               0x73eda753299d7d48ull};
static const uint64_t QINV_ = 0xfffffffeffffffffull;
static const uint64_t QR2_[4] = {0xc999e990f3f29c6dull, 0x2b6cedcb87925c23ull, 0x05d314967254398full,
                                 0x0748d9d99f59ff11ull};
static const uint64_t QONE_[4] = {0x00000001fffffffeull, 0x5884b7fa00034802ull, 0x998c4fefecbc4ff5ull,
                                  0x1824b159acc5056full};

template <int N, const uint64_t* M, const uint64_t* MINV, const uint64_t* MR2, const uint64_t* MONE>
struct Fe {
  uint64_t v[N];
  static Fe zero() { Fe r; memset(r.v, 0, sizeof r.v); return r; }
  static Fe one() { Fe r; memcpy(r.v, MONE, sizeof r.v); return r; }
  bool is_zero() const { uint64_t d = 0; for (int i = 0; i < N; i++) d |= v[i]; return !d; }
  bool operator==(const Fe& o) const { return !memcmp(v, o.v, sizeof v); }
  static bool geq(const uint64_t* a) {
    for (int i = N - 1; i >= 0; i--) if (a[i] != M[i]) return a[i] > M[i];
    return true;
  }
  static void subm(uint64_t* a) {
    uint64_t b = 0;
    for (int i = 0; i < N; i++) { u128 t = (u128)a[i] - M[i] - b; a[i] = (uint64_t)t; b = (uint64_t)(t >> 64) & 1; }
  }
  friend Fe operator+(const Fe& a, const Fe& b) {
    Fe r; uint64_t c = 0;
    for (int i = 0; i < N; i++) { u128 t = (u128)a.v[i] + b.v[i] + c; r.v[i] = (uint64_t)t; c = (uint64_t)(t >> 64); }
    if (c || geq(r.v)) subm(r.v);
    return r;
  }
  friend Fe operator-(const Fe& a, const Fe& b) {
    Fe r; uint64_t br = 0;
    for (int i = 0; i < N; i++) { u128 t = (u128)a.v[i] - b.v[i] - br; r.v[i] = (uint64_t)t; br = (uint64_t)(t >> 64) & 1; }
    if (br) { uint64_t c = 0; for (int i = 0; i < N; i++) { u128 t = (u128)r.v[i] + M[i] + c; r.v[i] = (uint64_t)t; c = (uint64_t)(t >> 64); } }
    return r;
  }
  friend Fe operator*(const Fe& a, const Fe& b) {
    uint64_t t[N + 2] = {0};
    for (int i = 0; i < N; i++) {
      uint64_t c = 0;
      for (int j = 0; j < N; j++) { u128 s = (u128)a.v[j] * b.v[i] + t[j] + c; t[j] = (uint64_t)s; c = (uint64_t)(s >> 64); }
      u128 s = (u128)t[N] + c; t[N] = (uint64_t)s; t[N + 1] = (uint64_t)(s >> 64);
      uint64_t m = t[0] * *MINV;
      s = (u128)m * M[0] + t[0]; c = (uint64_t)(s >> 64);
      for (int j = 1; j < N; j++) { s = (u128)m * M[j] + t[j] + c; t[j - 1] = (uint64_t)s; c = (uint64_t)(s >> 64); }
      s = (u128)t[N] + c; t[N - 1] = (uint64_t)s; t[N] = t[N + 1] + (uint64_t)(s >> 64);
    }
    Fe r; memcpy(r.v, t, sizeof r.v);
    if (t[N] || geq(r.v)) subm(r.v);
    return r;
  }
  Fe neg() const { return zero() - *this; }
  static Fe from_int(const uint64_t* x) { Fe a, r2; memcpy(a.v, x, sizeof a.v); memcpy(r2.v, MR2, sizeof r2.v); return a * r2; }
  void to_int(uint64_t* out) const { Fe o = zero(); o.v[0] = 1; Fe r = *this * o; memcpy(out, r.v, sizeof r.v); }
  Fe pow(const uint64_t* e, int words) const {
    Fe r = one();
    for (int i = words - 1; i >= 0; i--) for (int b = 63; b >= 0; b--) { r = r * r; if ((e[i] >> b) & 1) r = r * *this; }
    return r;
  }
  Fe inv() const { uint64_t e[N]; memcpy(e, M, sizeof e); e[0] -= 2; return pow(e, N); }
};
typedef Fe<6, P_, &PINV_, PR2_, PONE_> Fp;
typedef Fe<4, Q_, &QINV_, QR2_, QONE_> Fr;

struct Fp2 {
  Fp c0, c1;
  static Fp2 zero() { return {Fp::zero(), Fp::zero()}; }
  static Fp2 one() { return {Fp::one(), Fp::zero()}; }
  bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
  bool operator==(const Fp2& o) const { return c0 == o.c0 && c1 == o.c1; }
  friend Fp2 operator+(const Fp2& a, const Fp2& b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
  friend Fp2 operator-(const Fp2& a, const Fp2& b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
  friend Fp2 operator*(const Fp2& a, const Fp2& b) {
    Fp t0 = a.c0 * b.c0, t1 = a.c1 * b.c1;
    return {t0 - t1, (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1};
  }
  Fp2 neg() const { return {c0.neg(), c1.neg()}; }
  Fp2 inv() const { Fp t = (c0 * c0 + c1 * c1).inv(); return {c0 * t, (c1 * t).neg()}; }
};

// ===================================================================== curve (Jacobian)
template <class T>
struct Jac { T X, Y, Z; };
template <class T>
struct Aff { T x, y; bool inf; };

template <class T> static Jac<T> identity() { return {T::one(), T::one(), T::zero()}; }
template <class T>
static Jac<T> dbl(const Jac<T>& p) {
  if (p.Z.is_zero() || p.Y.is_zero()) return identity<T>();
  T A = p.X * p.X, B = p.Y * p.Y, C = B * B;
  T t = p.X + B;
  T D = t * t - A - C; D = D + D;
  T E = A + A + A, F = E * E;
  Jac<T> r;
  r.X = F - (D + D);
  T C8 = C + C; C8 = C8 + C8; C8 = C8 + C8;
  r.Y = E * (D - r.X) - C8;
  T yz = p.Y * p.Z; r.Z = yz + yz;
  return r;
}
template <class T>
static Jac<T> add(const Jac<T>& p, const Jac<T>& q) {
  if (p.Z.is_zero()) return q;
  if (q.Z.is_zero()) return p;
  T Z1Z1 = p.Z * p.Z, Z2Z2 = q.Z * q.Z;
  T U1 = p.X * Z2Z2, U2 = q.X * Z1Z1;
  T S1 = p.Y * q.Z * Z2Z2, S2 = q.Y * p.Z * Z1Z1;
  if (U1 == U2) { if (S1 == S2) return dbl(p); return identity<T>(); }
  T H = U2 - U1, HH = H + H, I = HH * HH, J = H * I;
  T r = S2 - S1; r = r + r;
  T V = U1 * I;
  Jac<T> o;
  o.X = r * r - J - (V + V);
  T S1J = S1 * J;
  o.Y = r * (V - o.X) - (S1J + S1J);
  T zz = p.Z + q.Z;
  o.Z = (zz * zz - Z1Z1 - Z2Z2) * H;
  return o;
}
// mixed addition (madd-2007-bl), q affine non-identity
template <class T>
static Jac<T> madd(const Jac<T>& p, const Aff<T>& q) {
  if (p.Z.is_zero()) return {q.x, q.y, T::one()};
  T Z1Z1 = p.Z * p.Z;
  T U2 = q.x * Z1Z1, S2 = q.y * p.Z * Z1Z1;
  if (U2 == p.X) { if (S2 == p.Y) return dbl(p); return identity<T>(); }
  T H = U2 - p.X, HH = H * H, I = HH + HH; I = I + I;
  T J = H * I, r = S2 - p.Y; r = r + r;
  T V = p.X * I;
  Jac<T> o;
  o.X = r * r - J - (V + V);
  T YJ = p.Y * J;
  o.Y = r * (V - o.X) - (YJ + YJ);
  T zh = p.Z + H;
  o.Z = zh * zh - Z1Z1 - HH;
  return o;
}
template <class T>
static Jac<T> mul(const Jac<T>& p, const uint64_t* k, int words) {
  Jac<T> acc = identity<T>();
  for (int i = words - 1; i >= 0; i--) for (int b = 63; b >= 0; b--) { acc = dbl(acc); if ((k[i] >> b) & 1) acc = add(acc, p); }
  return acc;
}
template <class T>
static Aff<T> to_affine(const Jac<T>& p) {
  if (p.Z.is_zero()) return {T::zero(), T::zero(), true};
  T zi = p.Z.inv(), zi2 = zi * zi;
  return {p.X * zi2, p.Y * zi2 * zi, false};
}
template <class T> static Jac<T> from_aff(const Aff<T>& a) { return a.inf ? identity<T>() : Jac<T>{a.x, a.y, T::one()}; }

// ===================================================================== encodings
static bool fp_be(const uint8_t* b, Fp* out, bool mask_flags) {
  uint64_t raw[6] = {0};
  for (int i = 0; i < 48; i++) {
    uint8_t x = b[i];
    if (i == 0 && mask_flags) x &= 0x1f;
    raw[(47 - i) / 8] |= (uint64_t)x << (8 * ((47 - i) % 8));
  }
  if (Fp::geq(raw)) return false;
  *out = Fp::from_int(raw);
  return true;
}
static void to_be(const Fp& a, uint8_t* out) {
  uint64_t raw[6];
  a.to_int(raw);
  for (int i = 0; i < 6; i++) for (int b = 0; b < 8; b++) out[47 - (8 * i + b)] = (uint8_t)(raw[i] >> (8 * b));
}
static bool lex_largest(const Fp& a) {
  uint64_t raw[6], half[6];
  a.to_int(raw);
  uint64_t c = 0;
  for (int i = 5; i >= 0; i--) { half[i] = (P_[i] >> 1) | c; c = P_[i] << 63; }
  for (int i = 5; i >= 0; i--) if (raw[i] != half[i]) return raw[i] > half[i];
  return false;
}
static bool read_g1(const uint8_t* b, Aff<Fp>* a) {
  if (b[0] & 0x40) { a->inf = true; a->x = a->y = Fp::zero(); return true; }
  a->inf = false;
  return fp_be(b, &a->x, true) && fp_be(b + 48, &a->y, false);
}
static bool read_g2(const uint8_t* b, Aff<Fp2>* a) {
  if (b[0] & 0x40) { a->inf = true; a->x = a->y = Fp2::zero(); return true; }
  a->inf = false;
  return fp_be(b, &a->x.c1, true) && fp_be(b + 48, &a->x.c0, false) && fp_be(b + 96, &a->y.c1, false) &&
         fp_be(b + 144, &a->y.c0, false);
}
static void g1_compressed(const Aff<Fp>& a, uint8_t* out) {
  if (a.inf) { memset(out, 0, 48); out[0] = 0xc0; return; }
  to_be(a.x, out); out[0] |= 0x80; if (lex_largest(a.y)) out[0] |= 0x20;
}
static void g2_compressed(const Aff<Fp2>& a, uint8_t* out) {
  if (a.inf) { memset(out, 0, 96); out[0] = 0xc0; return; }
  to_be(a.x.c1, out); to_be(a.x.c0, out + 48); out[0] |= 0x80;
  if (lex_largest(a.y.c1) || (a.y.c1.is_zero() && lex_largest(a.y.c0))) out[0] |= 0x20;
}

// ===================================================================== thread pool (rayon stand-in)
struct Pool {
  std::vector<std::thread> th;
  std::vector<std::function<void()>> q;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  size_t pending = 0;
  bool stop = false;
  int n;
  explicit Pool(int nthreads) : n(nthreads) {
    for (int i = 0; i < nthreads; i++)
      th.emplace_back([this] {
        for (;;) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [this] { return stop || !q.empty(); });
            if (stop && q.empty()) return;
            f = std::move(q.back());
            q.pop_back();
          }
          f();
          std::lock_guard<std::mutex> lk(mu);
          if (--pending == 0) done_cv.notify_all();
        }
      });
  }
  void spawn(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(mu);
    q.push_back(std::move(f));
    pending++;
    cv.notify_one();
  }
  void wait_all() {
    std::unique_lock<std::mutex> lk(mu);
    done_cv.wait(lk, [this] { return pending == 0; });
  }
  ~Pool() {
    { std::lock_guard<std::mutex> lk(mu); stop = true; }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  // Worker::scope chunking (multicore.rs:78-91)
  template <class F>
  void scope(size_t elements, F f) {
    size_t chunk = elements < (size_t)n ? 1 : elements / n;
    for (size_t s = 0; s < elements; s += chunk) {
      size_t e = std::min(elements, s + chunk);
      spawn([=] { f(s, e); });
    }
    wait_all();
  }
};

// ===================================================================== multiexp (multiexp.rs)
struct Fb { uint64_t w[4]; };  // FieldBits of Scalar::to_le_bits

template <class T>
struct MultiexpJob {
  const std::vector<Aff<T>>* bases;
  size_t offset;
  const std::vector<uint64_t>* density;  // nullptr = FullDensity
  const std::vector<Fb>* exps;
  int c;
  std::vector<Jac<T>> parts;
  std::atomic<int> err{0};
  Jac<T> result;
};

template <class T>
static void multiexp_window(MultiexpJob<T>* job, int widx) {
  const int c = job->c;
  const int skip = widx * c;
  const auto& bases = *job->bases;
  const auto& exps = *job->exps;
  Jac<T> acc = identity<T>();
  std::vector<Jac<T>> buckets((size_t)1 << c, identity<T>());
  size_t cur = job->offset;
  const bool handle_trivial = skip == 0;
  for (size_t i = 0; i < exps.size(); i++) {
    if (job->density && !(((*job->density)[i >> 6] >> (i & 63)) & 1)) continue;
    const uint64_t* e = exps[i].w;
    const bool rest_zero = !(e[1] | e[2] | e[3]) && (e[0] >> 1) == 0;
    const bool is_zero = rest_zero && !(e[0] & 1), is_one = rest_zero && (e[0] & 1);
    if (cur >= bases.size()) { job->err = 2; return; }  // skip()/next() at EOF
    if (is_zero) { cur++; continue; }
    if (is_one) {
      if (handle_trivial) { if (bases[cur].inf) { job->err = 1; return; } acc = madd(acc, bases[cur]); }
      cur++;
      continue;
    }
    uint64_t d = 0;  // bit-by-bit fold (multiexp.rs:208-214)
    for (int b = 0; b < c; b++) {
      int bit = skip + b;
      if (bit < 256 && ((e[bit >> 6] >> (bit & 63)) & 1)) d |= 1ull << b;
    }
    if (d) { if (bases[cur].inf) { job->err = 1; return; } buckets[d - 1] = madd(buckets[d - 1], bases[cur]); }
    cur++;
  }
  Jac<T> running = identity<T>();  // summation by parts (multiexp.rs:229-233)
  for (size_t k = buckets.size() - 1; k-- > 0;) {
    running = add(running, buckets[k]);
    acc = add(acc, running);
  }
  job->parts[widx] = acc;
}

template <class T>
static void multiexp_spawn(Pool& pool, MultiexpJob<T>* job) {
  size_t n = job->exps->size();
  job->c = n < 32 ? 3 : (int)ceil(log((double)(uint32_t)n));  // multiexp.rs:267-271
  int nw = (255 + job->c - 1) / job->c;
  job->parts.assign(nw, identity<T>());
  for (int w = 0; w < nw; w++) pool.spawn([job, w] { multiexp_window<T>(job, w); });
}
template <class T>
static void multiexp_finish(MultiexpJob<T>* job) {  // Horner (multiexp.rs:244-249)
  Jac<T> acc = identity<T>();
  for (size_t i = job->parts.size(); i-- > 0;) {
    for (int k = 0; k < job->c; k++) acc = dbl(acc);
    acc = add(acc, job->parts[i]);
  }
  job->result = acc;
}

// ===================================================================== domain (domain.rs)
static uint32_t bitrev(uint32_t n, int l) { uint32_t r = 0; for (int i = 0; i < l; i++) { r = (r << 1) | (n & 1); n >>= 1; } return r; }
static Fr fr_pow(const Fr& a, uint64_t e) { return a.pow(&e, 1); }

static void serial_fft(Fr* a, size_t n, const Fr& omega, int log_n) {
  for (uint32_t k = 0; k < n; k++) { uint32_t rk = bitrev(k, log_n); if (k < rk) std::swap(a[k], a[rk]); }
  size_t m = 1;
  for (int s = 0; s < log_n; s++) {
    Fr w_m = fr_pow(omega, n / (2 * m));
    for (size_t k = 0; k < n; k += 2 * m) {
      Fr w = Fr::one();
      for (size_t j = 0; j < m; j++) {
        Fr t = a[k + j + m] * w;
        a[k + j + m] = a[k + j] - t;
        a[k + j] = a[k + j] + t;
        w = w * w_m;
      }
    }
    m *= 2;
  }
}
static void parallel_fft(Pool& pool, Fr* a, size_t n, const Fr& omega, int log_n, int log_cpus) {
  const size_t num_cpus = (size_t)1 << log_cpus;
  const int log_new_n = log_n - log_cpus;
  std::vector<std::vector<Fr>> tmp(num_cpus, std::vector<Fr>((size_t)1 << log_new_n, Fr::zero()));
  const Fr new_omega = fr_pow(omega, num_cpus);
  for (size_t j = 0; j < num_cpus; j++) {
    pool.spawn([&, j] {
      Fr omega_j = fr_pow(omega, j);
      Fr omega_step = fr_pow(omega, (uint64_t)j << log_new_n);
      Fr elt = Fr::one();
      auto& t = tmp[j];
      for (size_t i = 0; i < t.size(); i++) {
        for (size_t s = 0; s < num_cpus; s++) {
          size_t idx = (i + (s << log_new_n)) % n;
          t[i] = t[i] + a[idx] * elt;
          elt = elt * omega_step;
        }
        elt = elt * omega_j;
      }
      serial_fft(t.data(), t.size(), new_omega, log_new_n);
    });
  }
  pool.wait_all();
  const size_t mask = num_cpus - 1;
  pool.scope(n, [&](size_t s, size_t e) { for (size_t idx = s; idx < e; idx++) a[idx] = tmp[idx & mask][idx >> log_cpus]; });
}
static void best_fft(Pool& pool, std::vector<Fr>& a, const Fr& omega, int log_n) {
  int log_cpus = 0;
  while ((2 << log_cpus) <= pool.n) log_cpus++;
  if (log_n <= log_cpus) serial_fft(a.data(), a.size(), omega, log_n);
  else parallel_fft(pool, a.data(), a.size(), omega, log_n, log_cpus);
}
static void scale_all(Pool& pool, std::vector<Fr>& a, const Fr& k) {
  pool.scope(a.size(), [&](size_t s, size_t e) { for (size_t i = s; i < e; i++) a[i] = a[i] * k; });
}
static void distribute_powers(Pool& pool, std::vector<Fr>& a, const Fr& g) {
  pool.scope(a.size(), [&](size_t s, size_t e) {
    Fr u = fr_pow(g, s);
    for (size_t i = s; i < e; i++) { a[i] = a[i] * u; u = u * g; }
  });
}

// ===================================================================== prover core (prover.rs:206-349)
struct Params {
  Aff<Fp> alpha_g1, beta_g1, delta_g1;
  Aff<Fp2> beta_g2, gamma_g2, delta_g2;
  std::vector<Aff<Fp>> ic, h, l, a, b_g1;
  std::vector<Aff<Fp2>> b_g2;
};
static bool parse_params(const uint8_t* p, size_t len, Params* out) {
  const uint8_t* end = p + len;
  auto take = [&](size_t n) -> const uint8_t* { if ((size_t)(end - p) < n) return nullptr; const uint8_t* r = p; p += n; return r; };
  auto u32 = [&](uint32_t* v) { const uint8_t* b = take(4); if (!b) return false; *v = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3]; return true; };
  const uint8_t* b;
  if (!(b = take(96)) || !read_g1(b, &out->alpha_g1)) return false;
  if (!(b = take(96)) || !read_g1(b, &out->beta_g1)) return false;
  if (!(b = take(192)) || !read_g2(b, &out->beta_g2)) return false;
  if (!(b = take(192)) || !read_g2(b, &out->gamma_g2)) return false;
  if (!(b = take(96)) || !read_g1(b, &out->delta_g1)) return false;
  if (!(b = take(192)) || !read_g2(b, &out->delta_g2)) return false;
  uint32_t n;
  if (!u32(&n)) return false;
  out->ic.resize(n);
  for (auto& x : out->ic) if (!(b = take(96)) || !read_g1(b, &x)) return false;
  for (auto* v : {&out->h, &out->l, &out->a, &out->b_g1}) {
    if (!u32(&n)) return false;
    v->resize(n);
    for (auto& x : *v) if (!(b = take(96)) || !read_g1(b, &x)) return false;
  }
  if (!u32(&n)) return false;
  out->b_g2.resize(n);
  for (auto& x : out->b_g2) if (!(b = take(192)) || !read_g2(b, &x)) return false;
  return true;
}

// splitmix64 / fr_stream (oracle/circuits.py)
static uint64_t splitmix64(uint64_t& st) {
  st += 0x9E3779B97F4A7C15ull;
  uint64_t z = st;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static std::vector<Fr> fr_stream(uint64_t seed, size_t count) {
  std::vector<Fr> out(count);
  uint64_t st = seed;
  for (auto& x : out) {
    uint64_t w[4];
    for (int k = 0; k < 4; k++) w[k] = splitmix64(st);
    while (Fr::geq(w)) Fr::subm(w);
    x = Fr::from_int(w);
  }
  return out;
}

struct Witness {
  std::vector<Fr> a, b, c, inputs, aux;
  std::vector<uint64_t> a_aux_d, b_in_d, b_aux_d;
};
static void set_bit(std::vector<uint64_t>& w, size_t i) { if (w.size() <= i / 64) w.resize(i / 64 + 1, 0); w[i >> 6] |= 1ull << (i & 63); }
// MiMC chain synthesis (mimc_mod.rs:50-129) + input constraints (prover.rs:198-204)
static void synthesize_chain(size_t rounds, uint64_t seed, Witness* w) {
  std::vector<Fr> consts = fr_stream(seed, rounds), pre = fr_stream(seed + 1, 2);
  w->inputs.push_back(Fr::one());
  Fr xl = pre[0], xr = pre[1];
  size_t xl_idx = 0, xr_idx = 1;
  bool xl_input = false;
  w->aux.push_back(xl); w->aux.push_back(xr);
  (void)xr_idx;
  for (size_t i = 0; i < rounds; i++) {
    Fr t = xl + consts[i], tmp = t * t;
    w->aux.push_back(tmp);
    size_t tmp_idx = w->aux.size() - 1;
    w->a.push_back(t); w->b.push_back(t); w->c.push_back(tmp);
    set_bit(w->a_aux_d, xl_idx); set_bit(w->b_aux_d, xl_idx); set_bit(w->b_in_d, 0);
    Fr nxl = t * tmp + xr;
    size_t nxl_idx;
    if (i == rounds - 1) { w->inputs.push_back(nxl); nxl_idx = 1; xl_input = true; }
    else { w->aux.push_back(nxl); nxl_idx = w->aux.size() - 1; }
    w->a.push_back(tmp); w->b.push_back(t); w->c.push_back(nxl - xr);
    set_bit(w->a_aux_d, tmp_idx); set_bit(w->b_aux_d, xl_idx); set_bit(w->b_in_d, 0);
    xr = xl; xl = nxl; xr_idx = xl_idx; xl_idx = nxl_idx;
  }
  (void)xl_input;
  for (size_t i = 0; i < w->inputs.size(); i++) { w->a.push_back(w->inputs[i]); w->b.push_back(Fr::zero()); w->c.push_back(Fr::zero()); }
  w->a_aux_d.resize((w->aux.size() + 63) / 64, 0);
  w->b_aux_d.resize((w->aux.size() + 63) / 64, 0);
  w->b_in_d.resize((w->inputs.size() + 63) / 64, 0);
}

static size_t popc(const std::vector<uint64_t>& w) { size_t c = 0; for (uint64_t x : w) c += __builtin_popcountll(x); return c; }
static std::vector<Fb> to_bits(const std::vector<Fr>& v, size_t n) {
  std::vector<Fb> out(n);
  for (size_t i = 0; i < n; i++) v[i].to_int(out[i].w);
  return out;
}

static int prove_core(Pool& pool, const Params& P, const Witness& W, const uint64_t r_c[4], const uint64_t s_c[4],
                      uint8_t out[192]) {
  size_t m = 1; int exp = 0;
  while (m < W.a.size()) { m *= 2; exp++; }
  uint64_t rou[4] = {0x3829971f439f0d2bull, 0xb63683508c2280b9ull, 0xd09b681922c813b4ull, 0x16a2a19edfe81f20ull};
  Fr omega = Fr::from_int(rou);
  for (int i = exp; i < 32; i++) omega = omega * omega;
  const Fr omegainv = omega.inv();
  uint64_t seven[4] = {7, 0, 0, 0}, mm[4] = {m, 0, 0, 0};
  const Fr g = Fr::from_int(seven), ginv = g.inv(), minv = Fr::from_int(mm).inv();
  std::vector<Fr> A(W.a), B(W.b), C(W.c);
  A.resize(m, Fr::zero()); B.resize(m, Fr::zero()); C.resize(m, Fr::zero());
  for (auto* v : {&A, &B, &C}) {  // ifft + coset_fft
    best_fft(pool, *v, omegainv, exp); scale_all(pool, *v, minv);
    distribute_powers(pool, *v, g); best_fft(pool, *v, omega, exp);
  }
  pool.scope(m, [&](size_t s, size_t e) { for (size_t i = s; i < e; i++) A[i] = A[i] * B[i] - C[i]; });
  const Fr zinv = (fr_pow(g, m) - Fr::one()).inv();
  scale_all(pool, A, zinv);
  best_fft(pool, A, omegainv, exp); scale_all(pool, A, minv); distribute_powers(pool, A, ginv);
  std::vector<Fb> h_bits = to_bits(A, m - 1);
  std::vector<Fb> in_bits = to_bits(W.inputs, W.inputs.size()), aux_bits = to_bits(W.aux, W.aux.size());
  const size_t ni = W.inputs.size();
  const size_t b_in_total = popc(W.b_in_d);
  MultiexpJob<Fp> jh, jl, jai, jaa, jbi, jba;
  MultiexpJob<Fp2> j2i, j2a;
  auto setup1 = [](MultiexpJob<Fp>& j, const std::vector<Aff<Fp>>* b, size_t off, const std::vector<uint64_t>* d, const std::vector<Fb>* e) { j.bases = b; j.offset = off; j.density = d; j.exps = e; };
  auto setup2 = [](MultiexpJob<Fp2>& j, const std::vector<Aff<Fp2>>* b, size_t off, const std::vector<uint64_t>* d, const std::vector<Fb>* e) { j.bases = b; j.offset = off; j.density = d; j.exps = e; };
  setup1(jh, &P.h, 0, nullptr, &h_bits);
  setup1(jl, &P.l, 0, nullptr, &aux_bits);
  setup1(jai, &P.a, 0, nullptr, &in_bits);
  setup1(jaa, &P.a, ni, &W.a_aux_d, &aux_bits);
  setup1(jbi, &P.b_g1, 0, &W.b_in_d, &in_bits);
  setup1(jba, &P.b_g1, b_in_total, &W.b_aux_d, &aux_bits);
  setup2(j2i, &P.b_g2, 0, &W.b_in_d, &in_bits);
  setup2(j2a, &P.b_g2, b_in_total, &W.b_aux_d, &aux_bits);
  // all 8 multiexps in flight together (Worker::compute), window tasks on one pool
  for (auto* j : {&jh, &jl, &jai, &jaa, &jbi, &jba}) multiexp_spawn(pool, j);
  for (auto* j : {&j2i, &j2a}) multiexp_spawn(pool, j);
  pool.wait_all();
  for (auto* j : {&jai, &jaa, &jbi, &jba, &jh, &jl}) { if (j->err) return j->err; multiexp_finish(j); }
  for (auto* j : {&j2i, &j2a}) { if (j->err) return j->err; multiexp_finish(j); }
  if (P.delta_g1.inf || P.delta_g2.inf) return 1;
  Fr r = Fr::from_int(r_c), s = Fr::from_int(s_c);
  uint64_t rs_c[4]; (r * s).to_int(rs_c);
  const Jac<Fp> d1 = from_aff(P.delta_g1), a1 = from_aff(P.alpha_g1), b1 = from_aff(P.beta_g1);
  const Jac<Fp2> d2 = from_aff(P.delta_g2), b2 = from_aff(P.beta_g2);
  Jac<Fp> g_a = add(mul(d1, r_c, 4), a1);
  Jac<Fp2> g_b = add(mul(d2, s_c, 4), b2);
  Jac<Fp> g_c = add(add(mul(d1, rs_c, 4), mul(a1, s_c, 4)), mul(b1, r_c, 4));
  Jac<Fp> a_ans = add(jai.result, jaa.result);
  g_a = add(g_a, a_ans);
  g_c = add(g_c, mul(a_ans, s_c, 4));
  Jac<Fp> b1_ans = add(jbi.result, jba.result);
  g_b = add(g_b, add(j2i.result, j2a.result));
  g_c = add(g_c, mul(b1_ans, r_c, 4));
  g_c = add(add(g_c, jh.result), jl.result);
  g1_compressed(to_affine(g_a), out);
  g2_compressed(to_affine(g_b), out + 48);
  g1_compressed(to_affine(g_c), out + 144);
  return 0;
}

extern "C" {

// Synthesize the MiMC chain (rounds, seed), then time `reps` prover-core runs
// (complete assignment -> proof) on `threads` threads.  params: Parameters::write
// bytes.  Returns 0 on success; *ms_core receives the median core time.
int bp_chain_prove(const uint8_t* params, size_t len, size_t rounds, uint64_t seed, int threads, int reps,
                   const uint64_t r[4], const uint64_t s[4], uint8_t proof_out[192], double* ms_core,
                   double* ms_synth) {
  Params P;
  if (!parse_params(params, len, &P)) return 11;
  auto t0 = std::chrono::steady_clock::now();
  Witness W;
  synthesize_chain(rounds, seed, &W);
  auto t1 = std::chrono::steady_clock::now();
  if (ms_synth) *ms_synth = std::chrono::duration<double, std::milli>(t1 - t0).count();
  Pool pool(threads > 0 ? threads : (int)std::thread::hardware_concurrency());
  std::vector<double> times;
  int st = 0;
  for (int i = 0; i < std::max(reps, 1); i++) {
    auto a = std::chrono::steady_clock::now();
    st = prove_core(pool, P, W, r, s, proof_out);
    auto b = std::chrono::steady_clock::now();
    if (st) return st;
    times.push_back(std::chrono::duration<double, std::milli>(b - a).count());
  }
  std::sort(times.begin(), times.end());
  if (ms_core) *ms_core = times[times.size() / 2];
  return 0;
}

int bp_hardware_threads(void) { return (int)std::thread::hardware_concurrency(); }

}  // extern "C"

static void write_uncompressed(const Aff<Fp>& a, uint8_t* out) {
  memset(out, 0, 96);
  if (a.inf) { out[0] = 0x40; return; }
  to_be(a.x, out);
  to_be(a.y, out + 48);
}
static void write_uncompressed(const Aff<Fp2>& a, uint8_t* out) {
  memset(out, 0, 192);
  if (a.inf) { out[0] = 0x40; return; }
  to_be(a.x.c1, out); to_be(a.x.c0, out + 48); to_be(a.y.c1, out + 96); to_be(a.y.c0, out + 144);
}

template <class T>
static int multiexp_host(const uint8_t* bases, size_t n_bases, size_t offset, const uint64_t* density_words,
                         const uint64_t* exps, size_t n, int threads, uint8_t* out, double* ms) {
  constexpr size_t PB = sizeof(T) == sizeof(Fp) ? 96 : 192;
  std::vector<Aff<T>> b(n_bases);
  for (size_t i = 0; i < n_bases; i++) {
    bool ok;
    if constexpr (PB == 96) ok = read_g1(bases + PB * i, &b[i]);
    else ok = read_g2(bases + PB * i, &b[i]);
    if (!ok) return 11;
  }
  std::vector<Fb> e(n);
  for (size_t i = 0; i < n; i++) memcpy(e[i].w, exps + 4 * i, 32);
  std::vector<uint64_t> dens;
  if (density_words) dens.assign(density_words, density_words + (n + 63) / 64);
  Pool pool(threads > 0 ? threads : (int)std::thread::hardware_concurrency());
  auto t0 = std::chrono::steady_clock::now();
  MultiexpJob<T> job;
  job.bases = &b;
  job.offset = offset;
  job.density = density_words ? &dens : nullptr;
  job.exps = &e;
  multiexp_spawn<T>(pool, &job);
  pool.wait_all();
  if (job.err) return job.err;
  multiexp_finish<T>(&job);
  auto t1 = std::chrono::steady_clock::now();
  if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  write_uncompressed(to_affine(job.result), out);
  return 0;
}

extern "C" {

// multiexp::multiexp (multiexp.rs:252-281) over G1 / G2 with bellman's schedule: one task per
// window on a pool of `threads`.  bases: n_bases uncompressed encodings (96 / 192 B);
// base_offset: the SourceBuilder's start index; density_words: QueryDensity bit words or NULL
// (FullDensity); exps: n canonical scalars (4 LE u64).  out: uncompressed result (0x40 flag =
// identity).  Returns 0, 1 (identity base), 2 (EOF) or 11 (bad encoding).
int bp_multiexp(int group, const uint8_t* bases, size_t n_bases, size_t base_offset, const uint64_t* density_words,
                const uint64_t* exps, size_t n, int threads, uint8_t* out, double* ms) {
  if (group == 1) return multiexp_host<Fp>(bases, n_bases, base_offset, density_words, exps, n, threads, out, ms);
  if (group == 2) return multiexp_host<Fp2>(bases, n_bases, base_offset, density_words, exps, n, threads, out, ms);
  return 10;
}

int bp_multiexp_g1(const uint8_t* bases, size_t n_bases, const uint64_t* exps, size_t n, int threads,
                   uint8_t out[96], double* ms) {
  return bp_multiexp(1, bases, n_bases, 0, nullptr, exps, n, threads, out, ms);
}

}  // extern "C"
