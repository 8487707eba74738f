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

static PyObject* drivers(PyObject* self, PyObject* args) {
  PyObject *rng, *rnd, *od_o, *sig_o, *sol_o, *terms_o, *out_o;
  double sigma, tod, sig, sol, wa, shc;
  Py_ssize_t n;
  long long s, dts;
  long month, day;
  unsigned long long tick0;
  (void)self;
  if (!PyArg_ParseTuple(args, "OOdnLLOOOllddOdddKO", &rng, &rnd, &sigma, &n, &s, &dts, &od_o, &sig_o, &sol_o, &month,
                        &day, &wa, &shc, &terms_o, &tod, &sig, &sol, &tick0, &out_o))
    return NULL;
  if (n < 0 || dts <= 0 || dts >= 86400 || s < -dts || s >= 86400) {
    PyErr_SetString(PyExc_ValueError, "drivers: bad tick count, time step or second of day");
    return NULL;
  }
  Py_buffer terms_b, od_b, sig_b, sol_b, out_b;
  const int solar_on = sol_o != Py_None;
  if (get_buf(terms_o, &terms_b, 3, 0, "terms") < 0) return NULL;
  if (get_buf(od_o, &od_b, 1440, 0, "od_tab") < 0) { PyBuffer_Release(&terms_b); return NULL; }
  if (get_buf(sig_o, &sig_b, 86400, 0, "sig_tab") < 0) {
    PyBuffer_Release(&terms_b); PyBuffer_Release(&od_b); return NULL;
  }
  if (solar_on && get_buf(sol_o, &sol_b, 1440, 1, "solar_tab") < 0) {
    PyBuffer_Release(&terms_b); PyBuffer_Release(&od_b); PyBuffer_Release(&sig_b); return NULL;
  }
  if (get_buf(out_o, &out_b, 4 * n, 1, "out") < 0) {
    PyBuffer_Release(&terms_b); PyBuffer_Release(&od_b); PyBuffer_Release(&sig_b);
    if (solar_on) PyBuffer_Release(&sol_b);
    return NULL;
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
  PyObject* gn = PyObject_GetAttrString(rng, "gauss_next");
  if (!gn) { err = 1; goto done; }
  if (gn != Py_None) {
    z = PyFloat_AsDouble(gn);
    have_z = 1;
    if (z == -1.0 && PyErr_Occurred()) { Py_DECREF(gn); err = 1; goto done; }
  }
  Py_DECREF(gn);

  Py_ssize_t k = 0;
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
  if (err) return NULL;
  return Py_BuildValue("nLddd", k, s, tod, sig, sol);
}

static PyMethodDef methods[] = {
    {"drivers", drivers, METH_VARARGS, "per-tick rollout drivers (see mdr_host.c)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_mdr_host", NULL, -1, methods};

PyMODINIT_FUNC PyInit__mdr_host(void) { return PyModule_Create(&module); }
