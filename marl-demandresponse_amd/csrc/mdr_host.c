/* mdr_host.c — the rollout's per-tick host drivers in C (CPython extension mdr_amd._mdr_host).
 *
 * Environment._driver_window_vec (mdr_amd/environment.py) for a constant base power and a flat /
 * sinusoidal / regular-steps signal: per tick (environment.py:86-106 of the reference,
 * server/app/core/environment/environment.py) the time advances by dt, the step uses the previous
 * outdoor temperature and the new datetime's solar gain, then one gauss(0, temp_std) draw gives
 * the new outdoor temperature (environment.py:132-159) and the new signal is read from the
 * second-of-day table (power_grid.py:80-161 via GridSignal.day_table).  The arithmetic is
 * CPython's, operation for operation (random.Random.gauss of Lib/random.py 3.10 with the
 * generator's own random() method and gauss_next cache; libm log / sqrt / cos / sin as the math
 * module calls them; IEEE double adds), so the mdr_tick rows are bit-identical to the Python loop
 * (tests/test_driver_window.py).  Compiled with -ffp-contract=off.
 *
 * rollout1(begin, rollout, ctx, stream, reward, rew_stride, p_dev, mode, sharded, <the driver arguments>):
 *   the same loop between mdr_rollout_begin and mdr_rollout (below).
 *
 * drivers(rng, random, sigma, n, s, dts, od_tab, sig_tab, solar_tab, month, day, window_area,
 *         shading_coeff, terms, tod, sig, sol, tick0, out) -> (k, s, tod, sig, sol)
 *   rng       the generator instance (its gauss_next attribute is read and written)
 *   random    its bound random() method
 *   s         seconds of the day before the first tick (>= -dts: the caller subtracts 86400 when
 *             a day ends); the run stops early (k < n) before a tick that crosses midnight, so the
 *             caller can switch to the next day's solar table
 *   od_tab    float64[1440]: od_temp without the draw, per minute of the day
 *   sig_tab   float64[86400]: the signal after a step, per second of the day
 *   solar_tab float64[1440] of the current (month, day), NaN = not computed yet (filled here by
 *             solar_minute below) or None when solar gain is off (solar 0.0)
 *   terms     float64[3 * T]: the CIBSE regression terms (coefficient, x power, y power)
 *   out       float64[n, 4] C-contiguous: t_od_prev, solar, s_prev, tick bits (mdr_tick rows)
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

static int get_buf(PyObject* o, Py_buffer* b, Py_ssize_t min_len, int writable, const char* what) {
  if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT | (writable ? PyBUF_WRITABLE : 0)) < 0) return -1;
  if (b->itemsize != 8 || !b->format || strcmp(b->format, "d") != 0 || b->len < min_len * 8) {
    PyBuffer_Release(b);
    PyErr_Format(PyExc_ValueError, "%s: expected a contiguous float64 buffer of >= %zd elements", what, min_len);
    return -1;
  }
  return 0;
}

/* drivers.py _solar_memo (compute_solar_gain, server/app/utils/utils.py:42-117): the same sum in
 * the same order; CPython's float ** int is libm pow for the non-negative bases here (x in
 * [0, 10], y >= 0), and the int 0 load outside daylight multiplies as 0.0 */
static double solar_minute(long month, long day, long hour, long minute, double wa, double shc,
                           const double* terms, Py_ssize_t nterms) {
  const double x = ((double)hour + (double)minute / 60.0) - 7.5;
  double load = 0.0;
  if (!(x < 0 || x > 10)) {
    const double y = ((double)month + (double)day / 30.0) - 1.0;
    load = terms[0];
    for (Py_ssize_t t = 1; t < nterms; ++t) {
      const double c = terms[3 * t], i = terms[3 * t + 1], j = terms[3 * t + 2];
      const double px = i == 1.0 ? x : pow(x, i), py = j == 1.0 ? y : pow(y, j);
      if (i != 0.0 && j != 0.0) load = load + px * py * c;
      else if (i != 0.0) load = load + px * c;
      else load = load + py * c;
    }
  }
  return wa * shc * load;
}

/* The driver loop of drivers() / rollout1(): parses the 19 driver arguments from `args` starting at
 * index `first`, fills `out`, and on success stores (k, s, tod, sig, sol) in *res. */
typedef struct {
  Py_ssize_t k, n;
  long long s;
  double tod, sig, sol;
  unsigned long long tick0;
  double* out;
} drv_res;

static int drivers_run(PyObject* args, Py_ssize_t first, drv_res* res) {
  PyObject *rng, *rnd, *od_o, *sig_o, *sol_o, *terms_o, *out_o;
  double sigma, tod, sig, sol, wa, shc;
  Py_ssize_t n;
  long long s, dts;
  long month, day;
  unsigned long long tick0;
  PyObject* sub = PyTuple_GetSlice(args, first, PyTuple_GET_SIZE(args));
  if (!sub) return -1;
  const int ok = PyArg_ParseTuple(sub, "OOdnLLOOOllddOdddKO", &rng, &rnd, &sigma, &n, &s, &dts, &od_o, &sig_o, &sol_o,
                                  &month, &day, &wa, &shc, &terms_o, &tod, &sig, &sol, &tick0, &out_o);
  Py_DECREF(sub);  /* (the parsed objects stay alive: `args` holds them) */
  if (!ok) return -1;
  if (n < 0 || dts <= 0 || dts >= 86400 || s < -dts || s >= 86400) {
    PyErr_SetString(PyExc_ValueError, "drivers: bad tick count, time step or second of day");
    return -1;
  }
  Py_buffer terms_b, od_b, sig_b, sol_b, out_b;
  const int solar_on = sol_o != Py_None;
  if (get_buf(terms_o, &terms_b, 3, 0, "terms") < 0) return -1;
  if (get_buf(od_o, &od_b, 1440, 0, "od_tab") < 0) { PyBuffer_Release(&terms_b); return -1; }
  if (get_buf(sig_o, &sig_b, 86400, 0, "sig_tab") < 0) {
    PyBuffer_Release(&terms_b); PyBuffer_Release(&od_b); return -1;
  }
  if (solar_on && get_buf(sol_o, &sol_b, 1440, 1, "solar_tab") < 0) {
    PyBuffer_Release(&terms_b); PyBuffer_Release(&od_b); PyBuffer_Release(&sig_b); return -1;
  }
  if (get_buf(out_o, &out_b, 4 * n, 1, "out") < 0) {
    PyBuffer_Release(&terms_b); PyBuffer_Release(&od_b); PyBuffer_Release(&sig_b);
    if (solar_on) PyBuffer_Release(&sol_b);
    return -1;
  }
  const double* terms = (const double*)terms_b.buf;
  const Py_ssize_t nterms = terms_b.len / 24;
  const double* od_tab = (const double*)od_b.buf;
  const double* sig_tab = (const double*)sig_b.buf;
  double* sol_tab = solar_on ? (double*)sol_b.buf : NULL;
  double* out = (double*)out_b.buf;
  const double two_pi = 2.0 * 3.141592653589793;  /* random.TWOPI = 2.0 * math.pi */

  /* the cached second normal deviate of random.gauss (None or a float) */
  double z = 0.0;
  int have_z = 0, err = 0;
  Py_ssize_t k = 0;
  PyObject* gn = PyObject_GetAttrString(rng, "gauss_next");
  if (!gn) { err = 1; goto done; }
  if (gn != Py_None) {
    z = PyFloat_AsDouble(gn);
    have_z = 1;
    if (z == -1.0 && PyErr_Occurred()) { Py_DECREF(gn); err = 1; goto done; }
  }
  Py_DECREF(gn);

  for (; k < n; ++k) {
    if (s + dts >= 86400) break;  /* the next tick is on the next day: the caller switches tables */
    s += dts;
    const long long m = s / 60;
    if (solar_on) {
      double v = sol_tab[m];
      if (v != v) {  /* first use of this minute of the day */
        v = solar_minute(month, day, (long)(m / 60), (long)(m % 60), wa, shc, terms, nterms);
        sol_tab[m] = v;
      }
      sol = v;
    }
    double* row = out + 4 * k;
    row[0] = tod;
    row[1] = sol;
    row[2] = sig;
    const uint64_t tk = (uint64_t)tick0 + (uint64_t)k;
    memcpy(&row[3], &tk, 8);
    /* random.gauss(0, sigma) */
    double g;
    if (have_z) {
      g = 0.0 + z * sigma;
      have_z = 0;
    } else {
      PyObject* r1 = PyObject_CallNoArgs(rnd);
      if (!r1) { err = 1; break; }
      const double u1 = PyFloat_AsDouble(r1);
      Py_DECREF(r1);
      PyObject* r2 = PyObject_CallNoArgs(rnd);
      if (!r2) { err = 1; break; }
      const double u2 = PyFloat_AsDouble(r2);
      Py_DECREF(r2);
      const double x2pi = u1 * two_pi;
      const double g2rad = sqrt(-2.0 * log(1.0 - u2));
      g = 0.0 + cos(x2pi) * g2rad * sigma;
      z = sin(x2pi) * g2rad;
      have_z = 1;
    }
    tod = od_tab[m] + g;
    sig = sig_tab[s];
  }
  if (!err) {
    PyObject* v = have_z ? PyFloat_FromDouble(z) : (Py_INCREF(Py_None), Py_None);
    if (!v || PyObject_SetAttrString(rng, "gauss_next", v) < 0) err = 1;
    Py_XDECREF(v);
  }
done:
  PyBuffer_Release(&terms_b);
  PyBuffer_Release(&od_b);
  PyBuffer_Release(&sig_b);
  if (solar_on) PyBuffer_Release(&sol_b);
  PyBuffer_Release(&out_b);
  if (err) return -1;
  res->k = k;
  res->n = n;
  res->s = s;
  res->tod = tod;
  res->sig = sig;
  res->sol = sol;
  res->tick0 = tick0;
  res->out = out;  /* (the caller's array, alive while `args` is) */
  return 0;
}

static PyObject* drivers(PyObject* self, PyObject* args) {
  (void)self;
  drv_res r;
  if (drivers_run(args, 0, &r) < 0) return NULL;
  return Py_BuildValue("nLddd", r.k, r.s, r.tod, r.sig, r.sol);
}

/* rollout1(begin, rollout, ctx, stream, reward, rew_stride, p_dev, mode, sharded, <the 19 driver arguments>)
 *   -> (rc_begin, rc_rollout, k, s, tod, sig, sol)
 * One short direct rollout (Environment.rollout's default sequence) without Python between its
 * steps: mdr_rollout_begin (the first window's count, before the drivers exist), the driver loop
 * into `out`, and — when the window did not stop at midnight (k == n) — mdr_rollout with those
 * ticks (no action buffer, no graph).  begin / rollout are the library's entry points (addresses
 * from ctypes); rc_rollout = ROLLOUT_NOT_CALLED (1: no library status is positive) when it was not
 * called (begin failed, or k < n: the caller finishes the driver window for the next day and
 * launches itself); any other value is mdr_rollout's own status (0, or a negative MDR_E*).
 * sharded != 0: `rollout` is mdr_rollout_sharded (a context with a communicator: begin also
 * allreduced the count, the KA step kernel is all that is left), called without use_graph. */
#define ROLLOUT_NOT_CALLED 1
typedef int (*begin_fn)(void* ctx, int n, uint64_t tick0, const uint8_t* action, int64_t act_stride, int mode,
                        void* stream);
typedef int (*rollout_fn)(void* ctx, int n, const void* ticks, const uint8_t* action, int64_t act_stride, int mode,
                          double* reward, int64_t rew_stride, double* p_out, int use_graph, void* stream);
typedef int (*rollout_sharded_fn)(void* ctx, int n, const void* ticks, const uint8_t* action, int64_t act_stride,
                                  int mode, double* reward, int64_t rew_stride, double* p_out, void* stream);

static PyObject* rollout1(PyObject* self, PyObject* args) {
  (void)self;
  if (PyTuple_GET_SIZE(args) != 9 + 19) {
    PyErr_SetString(PyExc_TypeError, "rollout1: 9 launch arguments + 19 driver arguments");
    return NULL;
  }
  unsigned long long a[9];
  for (int i = 0; i < 9; ++i) {
    a[i] = PyLong_AsUnsignedLongLongMask(PyTuple_GET_ITEM(args, i));
    if (PyErr_Occurred()) return NULL;
  }
  const begin_fn begin = (begin_fn)(uintptr_t)a[0];
  const rollout_fn roll = (rollout_fn)(uintptr_t)a[1];
  void* ctx = (void*)(uintptr_t)a[2];
  void* stream = (void*)(uintptr_t)a[3];
  double* reward = (double*)(uintptr_t)a[4];
  const int64_t rew_stride = (int64_t)a[5];
  double* p_dev = (double*)(uintptr_t)a[6];
  const int mode = (int)(int64_t)a[7];
  const int sharded = a[8] != 0;
  PyObject* n_o = PyTuple_GET_ITEM(args, 9 + 3);
  PyObject* t0_o = PyTuple_GET_ITEM(args, 9 + 17);
  const Py_ssize_t n = PyLong_AsSsize_t(n_o);
  const unsigned long long tick0 = PyLong_AsUnsignedLongLongMask(t0_o);
  if (PyErr_Occurred()) return NULL;
  if (!begin || !roll || !ctx || n < 1 || n > 0x7fffffff) {
    PyErr_SetString(PyExc_ValueError, "rollout1: bad launch arguments");
    return NULL;
  }
  const int rc_b = begin(ctx, (int)n, (uint64_t)tick0, NULL, 0, mode, stream);
  if (rc_b != 0) return Py_BuildValue("iinLddd", rc_b, ROLLOUT_NOT_CALLED, (Py_ssize_t)0, 0LL, 0.0, 0.0, 0.0);
  drv_res r;
  if (drivers_run(args, 9, &r) < 0) return NULL;
  int rc_r = ROLLOUT_NOT_CALLED;
  if (r.k == r.n)
    rc_r = sharded ? ((rollout_sharded_fn)(uintptr_t)a[1])(ctx, (int)n, r.out, NULL, 0, mode, reward, rew_stride, p_dev, stream)
                   : roll(ctx, (int)n, r.out, NULL, 0, mode, reward, rew_stride, p_dev, 0, stream);
  return Py_BuildValue("iinLddd", rc_b, rc_r, r.k, r.s, r.tod, r.sig, r.sol);
}

#ifndef MDR_HOST_SRC_HASH
#define MDR_HOST_SRC_HASH "unstamped"
#endif
/* build_id() -> the source hash build_ext.py stamped in (checked against the tree at import) */
static PyObject* build_id(PyObject* self, PyObject* args) {
  (void)self;
  (void)args;
  return PyUnicode_FromString("MDR_HOST_SRC_HASH:" MDR_HOST_SRC_HASH);
}

static PyMethodDef methods[] = {
    {"build_id", build_id, METH_NOARGS, "the source hash this extension was built from"},
    {"drivers", drivers, METH_VARARGS, "per-tick rollout drivers (see mdr_host.c)"},
    {"rollout1", rollout1, METH_VARARGS, "begin + drivers + mdr_rollout of one short rollout (see mdr_host.c)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_mdr_host", NULL, -1, methods};

PyMODINIT_FUNC PyInit__mdr_host(void) { return PyModule_Create(&module); }
