"""ORACLE (test infrastructure only) -- field-generic restatement of bellman's
Groth16 prover hot path.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this; the product (bellman-mpc_amd/) never does.

Every function cites the reference file:line it restates (paths relative to
/root/reference/bellman/src).  The restatement is generic over an `Engine` so
the same code runs on BLS12-381 (oracle.bls12_381) and on the reference's toy
DummyEngine (groth16/tests/dummy_engine.rs:331-365, Fr = Z/64513,
G1 = G2 = Fr), which is what pins it to the reference's own known-answer
constants (groth16/tests/mod.rs:342, 424-435, 574; see tests/test_oracle_kat.py).
"""
import math

from . import bls12_381 as bls


# ======================================================================= errors
class SynthesisError(Exception):
    """lib.rs:355-364"""
    code = -1


class UnexpectedIdentity(SynthesisError):
    code = 1   # multiexp.rs:63-65, prover.rs:309-313


class UnexpectedEof(SynthesisError):
    code = 2   # IoError(UnexpectedEof), multiexp.rs:55-61,74-80


class PolynomialDegreeTooLarge(SynthesisError):
    code = 3   # domain.rs:57-59


class DensitySizeMismatch(SynthesisError):
    code = 4   # the reference panics: multiexp.rs:277


class UnconstrainedVariable(SynthesisError):
    code = 5   # generator.rs:582-586


class AssignmentMissing(SynthesisError):
    code = 6


# ======================================================================= engines
class PrimeField:
    """Integer model of an ff::PrimeField (values kept canonical in [0, q))."""

    def __init__(self, q, S, generator, root_of_unity, num_bits):
        self.q = q
        self.S = S
        self.generator = generator
        self.root_of_unity = root_of_unity
        self.NUM_BITS = num_bits

    def inv(self, a):
        if a % self.q == 0:
            raise ZeroDivisionError
        return pow(a, self.q - 2, self.q)


class FieldGroup:
    """A prime field viewed as an additive group (DummyEngine's G1/G2/Gt)."""

    def __init__(self, q):
        self.q = q
        self.identity = 0

    def add(self, a, b):
        return (a + b) % self.q

    def double(self, a):
        return 2 * a % self.q

    def neg(self, a):
        return (-a) % self.q

    def mul(self, a, k):
        return a * k % self.q

    def is_identity(self, a):
        return a % self.q == 0

    def eq(self, a, b):
        return (a - b) % self.q == 0

    def to_affine(self, a):
        return a % self.q

    def from_affine(self, a):
        return a

    def add_affine(self, p, a):
        return (p + a) % self.q

    def affine_is_identity(self, a):
        return a % self.q == 0


class CurveGroup:
    """Adapter giving oracle.bls12_381.Curve the FieldGroup interface.
    Affine points are tuples or None (identity)."""

    def __init__(self, curve):
        self.c = curve
        self.identity = curve.identity

    def add(self, a, b):
        return self.c.add(a, b)

    def double(self, a):
        return self.c.double(a)

    def neg(self, a):
        return self.c.neg(a)

    def mul(self, a, k):
        return self.c.mul(a, k)

    def is_identity(self, a):
        return self.c.is_identity(a)

    def eq(self, a, b):
        return self.c.eq(a, b)

    def to_affine(self, a):
        return self.c.to_affine(a)

    def from_affine(self, a):
        return self.c.from_affine(a)

    def add_affine(self, p, a):
        return self.c.add_affine(p, a)

    def affine_is_identity(self, a):
        return a is None


class Engine:
    def __init__(self, name, fr, g1, g2, g1_gen, g2_gen):
        self.name = name
        self.Fr = fr
        self.G1 = g1
        self.G2 = g2
        self.g1_gen = g1_gen
        self.g2_gen = g2_gen


BLS12_381 = Engine(
    "bls12_381",
    PrimeField(bls.R, bls.FR_S, bls.FR_GENERATOR, bls.FR_ROOT_OF_UNITY, bls.FR_NUM_BITS),
    CurveGroup(bls.G1), CurveGroup(bls.G2),
    bls.G1.generator(), bls.G2.generator(),
)

# groth16/tests/dummy_engine.rs:15 (MODULUS_R = 64513), :289-317 (NUM_BITS 16, S 10,
# generator 5, root_of_unity 57751)
_DUMMY_R = 64513
DUMMY = Engine(
    "dummy",
    PrimeField(_DUMMY_R, 10, 5, 57751, 16),
    FieldGroup(_DUMMY_R), FieldGroup(_DUMMY_R),
    1, 1,
)


# ======================================================================= multiexp
def multiexp_window(n):
    """multiexp.rs:267-271 -- c = 3 if n < 32 else ceil(ln n)."""
    if n < 32:
        return 3
    return int(math.ceil(math.log(float(n))))


class _Source:
    """(Arc<Vec<G>>, usize) Source impl, multiexp.rs:45-86."""

    def __init__(self, G, bases, offset):
        self.G = G
        self.bases = bases
        self.i = offset

    def next(self):
        if len(self.bases) <= self.i:
            raise UnexpectedEof()
        b = self.bases[self.i]
        if self.G.affine_is_identity(b):
            raise UnexpectedIdentity()
        self.i += 1
        return b

    def skip(self, amt):
        if len(self.bases) <= self.i:
            raise UnexpectedEof()
        self.i += amt


def multiexp(engine, G, bases, offset, density, exponents, c=None):
    """multiexp.rs:159-281 restated.

    bases:     list of affine points (the SourceBuilder's Vec), consumed from `offset`
    density:   None (FullDensity) or list of bools (DensityTracker)
    exponents: list of canonical ints (Scalar::to_le_bits)
    Returns a projective point, or raises the SynthesisError the reference returns.
    """
    n = len(exponents)
    if c is None:
        c = multiexp_window(n)
    if density is not None and len(density) != n:
        raise DensitySizeMismatch()          # multiexp.rs:273-278 (assert)
    dens = density if density is not None else [True] * n
    mask = (1 << c) - 1

    def region(skip):                        # multiexp.rs:173-236
        acc = G.identity
        src = _Source(G, bases, offset)
        buckets = [G.identity] * ((1 << c) - 1)
        handle_trivial = skip == 0
        for exp, d in zip(exponents, dens):  # multiexp.rs:191-223
            if not d:
                continue
            if exp == 0:
                src.skip(1)
            elif exp == 1:
                if handle_trivial:
                    acc = G.add_affine(acc, src.next())
                else:
                    src.skip(1)
            else:
                digit = (exp >> skip) & mask
                if digit != 0:
                    buckets[digit - 1] = G.add_affine(buckets[digit - 1], src.next())
                else:
                    src.skip(1)
        running = G.identity                  # multiexp.rs:229-233
        for b in reversed(buckets):
            running = G.add(running, b)
            acc = G.add(acc, running)
        return acc

    parts = []
    for skip in range(0, engine.Fr.NUM_BITS, c):   # multiexp.rs:238-242
        try:
            parts.append((None, region(skip)))
        except SynthesisError as e:
            parts.append((e, None))
    acc = G.identity                          # multiexp.rs:244-249 (try_fold over rev)
    for err, part in reversed(parts):
        if err is not None:
            raise err
        for _ in range(c):
            acc = G.double(acc)
        acc = G.add(acc, part)
    return acc


def multiexp_naive(G, bases, offset, density, exponents):
    """Sum e_i * P_j over density-set i (bases consumed in order); the
    multiexp.rs:286-299 naive reference, extended with density."""
    acc = G.identity
    j = offset
    for i, e in enumerate(exponents):
        if density is not None and not density[i]:
            continue
        acc = G.add(acc, G.mul(G.from_affine(bases[j]), e))
        j += 1
    return acc


# ======================================================================= domain
def _bitreverse(n, l):
    r = 0
    for _ in range(l):
        r = (r << 1) | (n & 1)
        n >>= 1
    return r


def serial_fft(Fr, a, omega, log_n):
    """domain.rs:272-314 (in place, natural order out)."""
    q = Fr.q
    n = len(a)
    assert n == 1 << log_n
    for k in range(n):
        rk = _bitreverse(k, log_n)
        if k < rk:
            a[k], a[rk] = a[rk], a[k]
    m = 1
    for _ in range(log_n):
        w_m = pow(omega, n // (2 * m), q)
        k = 0
        while k < n:
            w = 1
            for j in range(m):
                t = a[k + j + m] * w % q
                a[k + j + m] = (a[k + j] - t) % q
                a[k + j] = (a[k + j] + t) % q
                w = w * w_m % q
            k += 2 * m
        m *= 2


def parallel_fft(Fr, a, omega, log_n, log_cpus):
    """domain.rs:316-372 (size-P DFT shuffle + sub-FFTs + transpose)."""
    q = Fr.q
    assert log_n >= log_cpus
    num_cpus = 1 << log_cpus
    log_new_n = log_n - log_cpus
    new_omega = pow(omega, num_cpus, q)
    tmp = [[0] * (1 << log_new_n) for _ in range(num_cpus)]
    for j in range(num_cpus):
        omega_j = pow(omega, j, q)
        omega_step = pow(omega, j << log_new_n, q)
        elt = 1
        t = tmp[j]
        for i in range(1 << log_new_n):
            for s in range(num_cpus):
                idx = (i + (s << log_new_n)) % (1 << log_n)
                t[i] = (t[i] + a[idx] * elt) % q
                elt = elt * omega_step % q
            elt = elt * omega_j % q
        serial_fft(Fr, t, new_omega, log_new_n)
    mask = num_cpus - 1
    for idx in range(len(a)):
        a[idx] = tmp[idx & mask][idx >> log_cpus]


def best_fft(Fr, a, omega, log_n, log_cpus=0):
    """domain.rs:261-269."""
    if log_n <= log_cpus:
        serial_fft(Fr, a, omega, log_n)
    else:
        parallel_fft(Fr, a, omega, log_n, log_cpus)


class EvaluationDomain:
    """domain.rs:21-190, over Scalar<Fr> coefficients (ints)."""

    def __init__(self, engine, coeffs, log_cpus=0):
        Fr = engine.Fr
        q = Fr.q
        m, exp = 1, 0
        while m < len(coeffs):                    # domain.rs:47-60
            m *= 2
            exp += 1
            if exp >= Fr.S:
                raise PolynomialDegreeTooLarge()
        omega = Fr.root_of_unity                  # domain.rs:62-66
        for _ in range(exp, Fr.S):
            omega = omega * omega % q
        self.Fr = Fr
        self.coeffs = [x % q for x in coeffs] + [0] * (m - len(coeffs))
        self.exp = exp
        self.omega = omega
        self.omegainv = Fr.inv(omega)
        self.geninv = Fr.inv(Fr.generator)
        self.minv = Fr.inv(m)
        self.log_cpus = log_cpus

    def __len__(self):
        return len(self.coeffs)

    def fft(self):                                # domain.rs:81-83
        best_fft(self.Fr, self.coeffs, self.omega, self.exp, self.log_cpus)

    def ifft(self):                               # domain.rs:85-99
        best_fft(self.Fr, self.coeffs, self.omegainv, self.exp, self.log_cpus)
        q = self.Fr.q
        self.coeffs = [v * self.minv % q for v in self.coeffs]

    def distribute_powers(self, g):               # domain.rs:101-113
        q = self.Fr.q
        u = 1
        for i in range(len(self.coeffs)):
            self.coeffs[i] = self.coeffs[i] * u % q
            u = u * g % q

    def coset_fft(self):                          # domain.rs:115-118
        self.distribute_powers(self.Fr.generator)
        self.fft()

    def icoset_fft(self):                         # domain.rs:120-125
        self.ifft()
        self.distribute_powers(self.geninv)

    def z(self, tau):                             # domain.rs:129-134
        return (pow(tau, len(self.coeffs), self.Fr.q) - 1) % self.Fr.q

    def divide_by_z_on_coset(self):               # domain.rs:139-151
        q = self.Fr.q
        i = self.Fr.inv(self.z(self.Fr.generator))
        self.coeffs = [v * i % q for v in self.coeffs]

    def mul_assign(self, other):                  # domain.rs:154-170
        assert len(self.coeffs) == len(other.coeffs)
        q = self.Fr.q
        self.coeffs = [a * b % q for a, b in zip(self.coeffs, other.coeffs)]

    def sub_assign(self, other):                  # domain.rs:173-189
        assert len(self.coeffs) == len(other.coeffs)
        q = self.Fr.q
        self.coeffs = [(a - b) % q for a, b in zip(self.coeffs, other.coeffs)]


# ======================================================================= R1CS API
class Variable:
    """lib.rs:212-236 (Variable(Index::Input|Aux(i)))."""
    __slots__ = ("kind", "index")

    def __init__(self, kind, index):
        self.kind = kind      # "input" | "aux"
        self.index = index

    def __repr__(self):
        return f"Variable({self.kind},{self.index})"


ONE = Variable("input", 0)   # ConstraintSystem::one(), lib.rs:434-436


class LinearCombination:
    """lib.rs:240-350.  `lc + var`, `lc - var`, `lc + (coeff, var)`,
    `lc + lc2`, `lc + (coeff, lc2)` as in the reference operator impls."""

    def __init__(self, terms=None):
        self.terms = list(terms or [])     # [(Variable, coeff)]

    @staticmethod
    def zero():
        return LinearCombination()

    def _push(self, var, coeff):
        return LinearCombination(self.terms + [(var, coeff)])

    def __add__(self, other):
        if isinstance(other, Variable):
            return self._push(other, 1)
        if isinstance(other, LinearCombination):
            return LinearCombination(self.terms + other.terms)
        coeff, x = other
        if isinstance(x, LinearCombination):
            return LinearCombination(self.terms + [(v, c * coeff) for v, c in x.terms])
        return self._push(x, coeff)

    def __sub__(self, other):
        if isinstance(other, Variable):
            return self._push(other, -1)
        if isinstance(other, LinearCombination):
            return LinearCombination(self.terms + [(v, -c) for v, c in other.terms])
        coeff, x = other
        if isinstance(x, LinearCombination):
            return LinearCombination(self.terms + [(v, -c * coeff) for v, c in x.terms])
        return self._push(x, -coeff)


class DensityTracker:
    """multiexp.rs:117-157."""

    def __init__(self):
        self.bv = []

    def add_element(self):
        self.bv.append(False)

    def inc(self, idx):
        self.bv[idx] = True

    def get_total_density(self):
        return sum(self.bv)


def _eval(q, lc, input_density, aux_density, inputs, aux):
    """prover.rs:19-53."""
    acc = 0
    for var, coeff in lc.terms:
        if var.kind == "input":
            tmp = inputs[var.index]
            if input_density is not None:
                input_density.inc(var.index)
        else:
            tmp = aux[var.index]
            if aux_density is not None:
                aux_density.inc(var.index)
        acc = (acc + tmp * coeff) % q
    return acc


class ProvingAssignment:
    """prover.rs:55-156."""

    def __init__(self, Fr):
        self.q = Fr.q
        self.a_aux_density = DensityTracker()
        self.b_input_density = DensityTracker()
        self.b_aux_density = DensityTracker()
        self.a, self.b, self.c = [], [], []
        self.input_assignment, self.aux_assignment = [], []

    @staticmethod
    def one():
        return ONE

    def alloc(self, name, f):
        v = f()
        if v is None:
            raise AssignmentMissing()
        self.aux_assignment.append(v % self.q)
        self.a_aux_density.add_element()
        self.b_aux_density.add_element()
        return Variable("aux", len(self.aux_assignment) - 1)

    def alloc_input(self, name, f):
        v = f()
        if v is None:
            raise AssignmentMissing()
        self.input_assignment.append(v % self.q)
        self.b_input_density.add_element()
        return Variable("input", len(self.input_assignment) - 1)

    def enforce(self, name, la, lb, lc):
        q = self.q
        z = LinearCombination.zero
        self.a.append(_eval(q, la(z()), None, self.a_aux_density,
                            self.input_assignment, self.aux_assignment))
        self.b.append(_eval(q, lb(z()), self.b_input_density, self.b_aux_density,
                            self.input_assignment, self.aux_assignment))
        self.c.append(_eval(q, lc(z()), None, None,
                            self.input_assignment, self.aux_assignment))

    def namespace(self, name):
        return self


class Params:
    """groth16/mod.rs:105-131 (VerifyingKey) + 224-247 (Parameters); affine points."""

    def __init__(self, vk, h, l, a, b_g1, b_g2):
        self.vk = vk          # dict alpha_g1 beta_g1 beta_g2 gamma_g2 delta_g1 delta_g2 ic
        self.h, self.l, self.a, self.b_g1, self.b_g2 = h, l, a, b_g1, b_g2


class Proof:
    def __init__(self, a, b, c):
        self.a, self.b, self.c = a, b, c   # affine


def synthesize_for_proving(engine, circuit):
    """prover.rs:187-204: assignment, circuit synthesis, x*0=0 input constraints."""
    prover = ProvingAssignment(engine.Fr)
    prover.alloc_input("", lambda: 1)
    circuit.synthesize(prover)
    for i in range(len(prover.input_assignment)):
        prover.enforce("", lambda lc, i=i: lc + Variable("input", i), lambda lc: lc, lambda lc: lc)
    return prover


def compute_h(engine, a, b, c, log_cpus=0):
    """prover.rs:210-231 H block: returns the m-1 coefficients of h (canonical)."""
    da = EvaluationDomain(engine, a, log_cpus)
    db = EvaluationDomain(engine, b, log_cpus)
    dc = EvaluationDomain(engine, c, log_cpus)
    da.ifft(); da.coset_fft()
    db.ifft(); db.coset_fft()
    dc.ifft(); dc.coset_fft()
    da.mul_assign(db)
    da.sub_assign(dc)
    da.divide_by_z_on_coset()
    da.icoset_fft()
    return da.coeffs[:len(da.coeffs) - 1]


def prove_from_assignment(engine, prover, params, r, s, log_cpus=0, naive=False):
    """prover.rs:206-349 given a complete ProvingAssignment."""
    Fr, G1, G2 = engine.Fr, engine.G1, engine.G2
    mexp = (lambda G, bases, off, dens, exps: multiexp_naive(G, bases, off, dens, exps)) if naive \
        else (lambda G, bases, off, dens, exps: multiexp(engine, G, bases, off, dens, exps))
    vk = params.vk
    h_coeffs = compute_h(engine, prover.a, prover.b, prover.c, log_cpus)
    h = mexp(G1, params.h, 0, None, h_coeffs)
    inputs = prover.input_assignment
    aux = prover.aux_assignment
    l = mexp(G1, params.l, 0, None, aux)
    a_inputs = mexp(G1, params.a, 0, None, inputs)
    a_aux = mexp(G1, params.a, len(inputs), prover.a_aux_density.bv, aux)
    b_in_total = prover.b_input_density.get_total_density()
    b_g1_inputs = mexp(G1, params.b_g1, 0, prover.b_input_density.bv, inputs)
    b_g1_aux = mexp(G1, params.b_g1, b_in_total, prover.b_aux_density.bv, aux)
    b_g2_inputs = mexp(G2, params.b_g2, 0, prover.b_input_density.bv, inputs)
    b_g2_aux = mexp(G2, params.b_g2, b_in_total, prover.b_aux_density.bv, aux)
    if G1.affine_is_identity(vk["delta_g1"]) or G2.affine_is_identity(vk["delta_g2"]):
        raise UnexpectedIdentity()                         # prover.rs:309-313
    d1 = G1.from_affine(vk["delta_g1"])
    d2 = G2.from_affine(vk["delta_g2"])
    g_a = G1.add_affine(G1.mul(d1, r), vk["alpha_g1"])     # prover.rs:315-316
    g_b = G2.add_affine(G2.mul(d2, s), vk["beta_g2"])      # prover.rs:317-318
    rs = r * s % Fr.q
    g_c = G1.mul(d1, rs)                                   # prover.rs:321-327
    g_c = G1.add(g_c, G1.mul(G1.from_affine(vk["alpha_g1"]), s))
    g_c = G1.add(g_c, G1.mul(G1.from_affine(vk["beta_g1"]), r))
    a_answer = G1.add(a_inputs, a_aux)                     # prover.rs:328-332
    g_a = G1.add(g_a, a_answer)
    a_answer = G1.mul(a_answer, s)
    g_c = G1.add(g_c, a_answer)
    b1_answer = G1.add(b_g1_inputs, b_g1_aux)              # prover.rs:334-341
    b2_answer = G2.add(b_g2_inputs, b_g2_aux)
    g_b = G2.add(g_b, b2_answer)
    b1_answer = G1.mul(b1_answer, r)
    g_c = G1.add(g_c, b1_answer)
    g_c = G1.add(g_c, h)                                   # prover.rs:342-343
    g_c = G1.add(g_c, l)
    return Proof(G1.to_affine(g_a), G2.to_affine(g_b), G1.to_affine(g_c))


def create_proof(engine, circuit, params, r, s, log_cpus=0, naive=False):
    """prover.rs:175-350."""
    prover = synthesize_for_proving(engine, circuit)
    return prove_from_assignment(engine, prover, params, r, s, log_cpus, naive)


def create_random_proof(engine, circuit, params, rng=None, **kw):
    """prover.rs:158-173 -- the fork ignores rng: r = 27134, s = 17146."""
    return create_proof(engine, circuit, params, 27134, 17146, **kw)


def proof_to_bytes(proof):
    """Proof::write, groth16/mod.rs:42-48 (BLS12-381 only): A(48) || B(96) || C(48)."""
    return (bls.g1_to_compressed(proof.a) + bls.g2_to_compressed(proof.b)
            + bls.g1_to_compressed(proof.c))


# ======================================================================= generator
class KeypairAssembly:
    """generator.rs:44-156."""

    def __init__(self):
        self.num_inputs = 0
        self.num_aux = 0
        self.num_constraints = 0
        self.at_inputs, self.bt_inputs, self.ct_inputs = [], [], []
        self.at_aux, self.bt_aux, self.ct_aux = [], [], []

    @staticmethod
    def one():
        return ONE

    def alloc(self, name, f):
        idx = self.num_aux
        self.num_aux += 1
        self.at_aux.append([]); self.bt_aux.append([]); self.ct_aux.append([])
        return Variable("aux", idx)

    def alloc_input(self, name, f):
        idx = self.num_inputs
        self.num_inputs += 1
        self.at_inputs.append([]); self.bt_inputs.append([]); self.ct_inputs.append([])
        return Variable("input", idx)

    def enforce(self, name, la, lb, lc):
        z = LinearCombination.zero
        for lcx, ins, auxs in ((la(z()), self.at_inputs, self.at_aux),
                               (lb(z()), self.bt_inputs, self.bt_aux),
                               (lc(z()), self.ct_inputs, self.ct_aux)):
            for var, coeff in lcx.terms:
                (ins if var.kind == "input" else auxs)[var.index].append((coeff, self.num_constraints))
        self.num_constraints += 1

    def namespace(self, name):
        return self


def generate_parameters(engine, circuit, alpha, beta, gamma, delta, tau, g1=None, g2=None):
    """Upstream classic CRS generation, generator.rs:241-572 + 614-633,
    WITHOUT the fork's MPC consistency asserts (generator.rs:298-308, 573-611),
    which only hold for 4-constraint circuits."""
    Fr, G1, G2 = engine.Fr, engine.G1, engine.G2
    q = Fr.q
    g1 = engine.g1_gen if g1 is None else g1
    g2 = engine.g2_gen if g2 is None else g2
    asm = KeypairAssembly()
    asm.alloc_input("", lambda: 1)
    circuit.synthesize(asm)
    for i in range(asm.num_inputs):
        asm.enforce("", lambda lc, i=i: lc + Variable("input", i), lambda lc: lc, lambda lc: lc)
    dom = EvaluationDomain(engine, [0] * asm.num_constraints)
    m = len(dom.coeffs)
    gamma_inv = Fr.inv(gamma)
    delta_inv = Fr.inv(delta)
    powers = [pow(tau, i, q) for i in range(m)]
    coeff = dom.z(tau) * delta_inv % q
    h = [G1.to_affine(G1.mul(g1, powers[i] * coeff % q)) for i in range(m - 1)]
    dom.coeffs = powers
    dom.ifft()
    lag = dom.coeffs

    def eval_at_tau(terms):
        acc = 0
        for c, idx in terms:
            acc = (acc + lag[idx] * c) % q
        return acc

    def evaluate(at, bt, ct, inv):
        a, b_g1, b_g2, ext = [], [], [], []
        for at_i, bt_i, ct_i in zip(at, bt, ct):
            av = eval_at_tau(at_i)
            bv = eval_at_tau(bt_i)
            cv = eval_at_tau(ct_i)
            a.append(G1.to_affine(G1.mul(g1, av)) if av else G1.to_affine(G1.identity))
            if bv:
                b_g1.append(G1.to_affine(G1.mul(g1, bv)))
                b_g2.append(G2.to_affine(G2.mul(g2, bv)))
            else:
                b_g1.append(G1.to_affine(G1.identity))
                b_g2.append(G2.to_affine(G2.identity))
            e = (av * beta + bv * alpha + cv) * inv % q
            ext.append(G1.to_affine(G1.mul(g1, e)))
        return a, b_g1, b_g2, ext

    a_in, b1_in, b2_in, ic = evaluate(asm.at_inputs, asm.bt_inputs, asm.ct_inputs, gamma_inv)
    a_ax, b1_ax, b2_ax, l = evaluate(asm.at_aux, asm.bt_aux, asm.ct_aux, delta_inv)
    for e in l:
        if G1.affine_is_identity(e):
            raise UnconstrainedVariable()
    vk = dict(
        alpha_g1=G1.to_affine(G1.mul(g1, alpha)),
        beta_g1=G1.to_affine(G1.mul(g1, beta)),
        beta_g2=G2.to_affine(G2.mul(g2, beta)),
        gamma_g2=G2.to_affine(G2.mul(g2, gamma)),
        delta_g1=G1.to_affine(G1.mul(g1, delta)),
        delta_g2=G2.to_affine(G2.mul(g2, delta)),
        ic=ic,
    )
    keep = lambda G, xs: [x for x in xs if not G.affine_is_identity(x)]
    return Params(vk, h, l, keep(G1, a_in + a_ax), keep(G1, b1_in + b1_ax), keep(G2, b2_in + b2_ax))


# Fixed toxic waste of the fork's generate_random_parameters (generator.rs:32-38)
FORK_TOXIC = dict(alpha=6, beta=24, gamma=6, delta=24, tau=2)


def generate_random_parameters(engine, circuit):
    """generator.rs:21-40 (fixed alpha=6, beta=24, gamma=6, delta=24, tau=2)."""
    return generate_parameters(engine, circuit, **FORK_TOXIC)


# ======================================================================= DummyEngine verifier
def verify_dummy(engine, params, proof, public_inputs):
    """verifier.rs:23-62 specialised to DummyEngine, where the pairing e(a,b)
    is the field product (dummy_engine.rs:344-364):
    A*B == alpha*beta + IC(x)*gamma + C*delta."""
    q = engine.Fr.q
    vk = params.vk
    acc = vk["ic"][0]
    for x, b in zip(public_inputs, vk["ic"][1:]):
        acc = (acc + b * x) % q
    lhs = proof.a * proof.b % q
    rhs = (vk["alpha_g1"] * vk["beta_g2"] + acc * vk["gamma_g2"] + proof.c * vk["delta_g2"]) % q
    return lhs == rhs


# ======================================================================= Parameters::write
def params_to_bytes(params):
    """Parameters::write (groth16/mod.rs:260-290) incl. VerifyingKey::write (145-159);
    BLS12-381 only, uncompressed encodings."""
    vk = params.vk
    out = bytearray()
    out += bls.g1_to_uncompressed(vk["alpha_g1"])
    out += bls.g1_to_uncompressed(vk["beta_g1"])
    out += bls.g2_to_uncompressed(vk["beta_g2"])
    out += bls.g2_to_uncompressed(vk["gamma_g2"])
    out += bls.g1_to_uncompressed(vk["delta_g1"])
    out += bls.g2_to_uncompressed(vk["delta_g2"])
    out += len(vk["ic"]).to_bytes(4, "big")
    for p in vk["ic"]:
        out += bls.g1_to_uncompressed(p)
    for vec, enc in ((params.h, bls.g1_to_uncompressed), (params.l, bls.g1_to_uncompressed),
                     (params.a, bls.g1_to_uncompressed), (params.b_g1, bls.g1_to_uncompressed),
                     (params.b_g2, bls.g2_to_uncompressed)):
        out += len(vec).to_bytes(4, "big")
        for p in vec:
            out += enc(p)
    return bytes(out)
