/* Bulk construction of the Python objects Tagger.tag_batch returns
 * (CPython C API, module `_ltpy`).
 *
 * The decoder's results are a few int32 codes per path node; the reference
 * API hands back `Sequence`s of `Word` namedtuples (`beam/beam.py:88-116`,
 * `dictionary/dictionary.py:169-199`).  Building 1-2 million Word tuples per
 * 64K sentences through `map(tuple.__new__, zip(...))` held the caller's
 * thread for most of the pipeline's time (tools/prof_materialise.py).  Here
 * the tuples are allocated by the Word type itself (a tuple subclass without
 * a __dict__, as tuple.__new__ does for subclasses) and filled with shared
 * references to the already decoded field strings, and the path lists are
 * cut in one pass.
 *
 *   words(word_type, out, pos, uniq, codes, ints)
 *       out[pos[i]] = word_type(uniq[f][codes[f][i]] for f in 0..4 (code -1 -> None),
 *                               len[i], b[i], e[i], bool(is_l[i]))
 *   unknowns(word_type, out, pos, chars, sent, b, d, unk_tag)
 *       out[pos[i]] = word_type(sub, sub, None, unk_tag, None, d, b, b + d, False),
 *                     sub = chars[sent[i]][b[i]:b[i] + d[i]]
 *   unknowns_cp(word_type, out, pos, cps, off, sent, b, d, unk_tag)
 *       as unknowns, sub = the code points cps[off[sent[i]] + b[i] .. + d[i]) as a str
 *   scatter(out, pos, vals)      out[pos[i]] = vals[i]
 *   paths(flat, ends, bos, eos, has)
 *       [[bos] + flat[ends[s-1]:ends[s]] + [eos[s]]  if has[s] else None  for s]
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

typedef struct {
  Py_buffer b;
  int ok;
} Buf;

/* A C-contiguous buffer of >= n items of itemsize bytes (numpy arrays made
 * by the caller with the dtype named in the module doc). */
static int get_buf(PyObject* o, Buf* B, Py_ssize_t itemsize, Py_ssize_t n, const char* what) {
  B->ok = 0;
  if (PyObject_GetBuffer(o, &B->b, PyBUF_C_CONTIGUOUS) < 0) return -1;
  B->ok = 1;
  if (B->b.itemsize != itemsize || B->b.len / itemsize < n) {
    PyErr_Format(PyExc_ValueError, "_ltpy: %s: wrong item size or too short", what);
    return -1;
  }
  return 0;
}

static void rel(Buf* B) {
  if (B->ok) PyBuffer_Release(&B->b);
  B->ok = 0;
}

/* A new instance of the tuple subclass `tp` with n items (all NULL). */
static PyObject* new_tuple(PyTypeObject* tp, Py_ssize_t n) {
  return tp->tp_alloc(tp, n);
}

/* A filled Word holds only str / int / bool / None, so it can never be part
 * of a reference cycle.  CPython untracks such tuples during a collection
 * only for exact tuples (gcmodule.c untrack_tuples), never for subclasses:
 * left tracked, the 1-2 million Words of a 64K-sentence call stay on the
 * collector's lists and every full collection after the call walks them
 * (~0.15 s at 64K sentences, one call in three or four).  Untrack it here
 * when every item is a non-container. */
static void untrack_atomic(PyObject* w) {
  const Py_ssize_t n = PyTuple_GET_SIZE(w);
  for (Py_ssize_t i = 0; i < n; ++i)
    if (PyObject_IS_GC(PyTuple_GET_ITEM(w, i))) return;
  PyObject_GC_UnTrack(w);
}

static int check_word_type(PyObject* t) {
  if (!PyType_Check(t) || !PyType_IsSubtype((PyTypeObject*)t, &PyTuple_Type) ||
      ((PyTypeObject*)t)->tp_dictoffset != 0) {
    PyErr_SetString(PyExc_TypeError, "_ltpy: word_type must be a tuple subclass without __dict__");
    return -1;
  }
  return 0;
}

static PyObject* py_words(PyObject* self, PyObject* args) {
  PyObject *wt, *out, *pos_o, *uniq, *codes, *ints;
  if (!PyArg_ParseTuple(args, "OO!OO!O!O!", &wt, &PyList_Type, &out, &pos_o, &PyTuple_Type, &uniq, &PyTuple_Type,
                        &codes, &PyTuple_Type, &ints))
    return NULL;
  if (check_word_type(wt) < 0) return NULL;
  if (PyTuple_GET_SIZE(uniq) != 5 || PyTuple_GET_SIZE(codes) != 5 || PyTuple_GET_SIZE(ints) != 4) {
    PyErr_SetString(PyExc_ValueError, "_ltpy.words: 5 string fields and 4 integer fields");
    return NULL;
  }
  Buf pos, cb[5], ib[4];
  memset(cb, 0, sizeof cb);
  memset(ib, 0, sizeof ib);
  pos.ok = 0;
  PyObject* res = NULL;
  Py_ssize_t n;
  {
    if (PyObject_GetBuffer(pos_o, &pos.b, PyBUF_C_CONTIGUOUS) < 0) return NULL;
    pos.ok = 1;
    if (pos.b.itemsize != 8) {
      PyErr_SetString(PyExc_ValueError, "_ltpy.words: pos must be int64");
      goto done;
    }
    n = pos.b.len / 8;
  }
  for (int f = 0; f < 5; ++f) {
    if (!PyList_Check(PyTuple_GET_ITEM(uniq, f))) {
      PyErr_SetString(PyExc_TypeError, "_ltpy.words: uniq fields must be lists");
      goto done;
    }
    if (get_buf(PyTuple_GET_ITEM(codes, f), &cb[f], 4, n, "codes") < 0) goto done;
  }
  for (int f = 0; f < 4; ++f)
    if (get_buf(PyTuple_GET_ITEM(ints, f), &ib[f], f == 3 ? 1 : 8, n, "ints") < 0) goto done;
  {
    const int64_t* P = (const int64_t*)pos.b.buf;
    const Py_ssize_t nout = PyList_GET_SIZE(out);
    Py_ssize_t nu[5];
    PyObject** U[5];
    for (int f = 0; f < 5; ++f) {
      PyObject* l = PyTuple_GET_ITEM(uniq, f);
      nu[f] = PyList_GET_SIZE(l);
      U[f] = ((PyListObject*)l)->ob_item;
    }
    /* validate every index first: the fill below cannot fail half-way */
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (P[i] < 0 || P[i] >= nout) {
        PyErr_SetString(PyExc_IndexError, "_ltpy.words: position out of range");
        goto done;
      }
      for (int f = 0; f < 5; ++f) {
        const int32_t c = ((const int32_t*)cb[f].b.buf)[i];
        if (c < -1 || c >= nu[f]) {
          PyErr_SetString(PyExc_IndexError, "_ltpy.words: string code out of range");
          goto done;
        }
      }
    }
    const int64_t* L = (const int64_t*)ib[0].b.buf;
    const int64_t* B = (const int64_t*)ib[1].b.buf;
    const int64_t* E = (const int64_t*)ib[2].b.buf;
    const uint8_t* IL = (const uint8_t*)ib[3].b.buf;
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* w = new_tuple((PyTypeObject*)wt, 9);
      if (!w) goto done;
      for (int f = 0; f < 5; ++f) {
        const int32_t c = ((const int32_t*)cb[f].b.buf)[i];
        PyObject* s = c < 0 ? Py_None : U[f][c];
        Py_INCREF(s);
        PyTuple_SET_ITEM(w, f, s);
      }
      PyObject *ln = PyLong_FromLongLong(L[i]), *bb = PyLong_FromLongLong(B[i]), *ee = PyLong_FromLongLong(E[i]);
      if (!ln || !bb || !ee) {
        Py_XDECREF(ln);
        Py_XDECREF(bb);
        Py_XDECREF(ee);
        Py_DECREF(w);
        goto done;
      }
      PyTuple_SET_ITEM(w, 5, ln);
      PyTuple_SET_ITEM(w, 6, bb);
      PyTuple_SET_ITEM(w, 7, ee);
      PyObject* il = IL[i] ? Py_True : Py_False;
      Py_INCREF(il);
      PyTuple_SET_ITEM(w, 8, il);
      untrack_atomic(w);
      PyList_SetItem(out, P[i], w); /* steals w, releases the old item */
    }
  }
  Py_INCREF(Py_None);
  res = Py_None;
done:
  rel(&pos);
  for (int f = 0; f < 5; ++f) rel(&cb[f]);
  for (int f = 0; f < 4; ++f) rel(&ib[f]);
  return res;
}

static PyObject* py_unknowns(PyObject* self, PyObject* args) {
  PyObject *wt, *out, *pos_o, *chars, *sent_o, *b_o, *d_o, *unk;
  if (!PyArg_ParseTuple(args, "OO!OO!OOOO", &wt, &PyList_Type, &out, &pos_o, &PyList_Type, &chars, &sent_o, &b_o,
                        &d_o, &unk))
    return NULL;
  if (check_word_type(wt) < 0) return NULL;
  Buf pos = {0}, sb = {0}, bb = {0}, db = {0};
  PyObject* res = NULL;
  Py_ssize_t n;
  if (PyObject_GetBuffer(pos_o, &pos.b, PyBUF_C_CONTIGUOUS) < 0) return NULL;
  pos.ok = 1;
  if (pos.b.itemsize != 8) {
    PyErr_SetString(PyExc_ValueError, "_ltpy.unknowns: pos must be int64");
    goto done;
  }
  n = pos.b.len / 8;
  if (get_buf(sent_o, &sb, 8, n, "sent") < 0 || get_buf(b_o, &bb, 8, n, "b") < 0 ||
      get_buf(d_o, &db, 8, n, "d") < 0)
    goto done;
  {
    const int64_t *P = (const int64_t*)pos.b.buf, *S = (const int64_t*)sb.b.buf, *Bg = (const int64_t*)bb.b.buf,
                  *D = (const int64_t*)db.b.buf;
    const Py_ssize_t nout = PyList_GET_SIZE(out), ns = PyList_GET_SIZE(chars);
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (P[i] < 0 || P[i] >= nout || S[i] < 0 || S[i] >= ns || Bg[i] < 0 || D[i] < 1) {
        PyErr_SetString(PyExc_IndexError, "_ltpy.unknowns: index out of range");
        goto done;
      }
      PyObject* ch = PyList_GET_ITEM(chars, S[i]);
      if (!PyUnicode_Check(ch) || Bg[i] + D[i] > PyUnicode_GET_LENGTH(ch)) {
        PyErr_SetString(PyExc_IndexError, "_ltpy.unknowns: span outside the sentence");
        goto done;
      }
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* sub = PyUnicode_Substring(PyList_GET_ITEM(chars, S[i]), Bg[i], Bg[i] + D[i]);
      if (!sub) goto done;
      PyObject* w = new_tuple((PyTypeObject*)wt, 9);
      PyObject *ln = PyLong_FromLongLong(D[i]), *b0 = PyLong_FromLongLong(Bg[i]),
               *e0 = PyLong_FromLongLong(Bg[i] + D[i]);
      if (!w || !ln || !b0 || !e0) {
        Py_DECREF(sub);
        Py_XDECREF(w);
        Py_XDECREF(ln);
        Py_XDECREF(b0);
        Py_XDECREF(e0);
        goto done;
      }
      Py_INCREF(sub);
      PyTuple_SET_ITEM(w, 0, sub);
      PyTuple_SET_ITEM(w, 1, sub);
      Py_INCREF(Py_None);
      PyTuple_SET_ITEM(w, 2, Py_None);
      Py_INCREF(unk);
      PyTuple_SET_ITEM(w, 3, unk);
      Py_INCREF(Py_None);
      PyTuple_SET_ITEM(w, 4, Py_None);
      PyTuple_SET_ITEM(w, 5, ln);
      PyTuple_SET_ITEM(w, 6, b0);
      PyTuple_SET_ITEM(w, 7, e0);
      Py_INCREF(Py_False);
      PyTuple_SET_ITEM(w, 8, Py_False);
      untrack_atomic(w);
      PyList_SetItem(out, P[i], w);
    }
  }
  Py_INCREF(Py_None);
  res = Py_None;
done:
  rel(&pos);
  rel(&sb);
  rel(&bb);
  rel(&db);
  return res;
}

static PyObject* py_unknowns_cp(PyObject* self, PyObject* args) {
  PyObject *wt, *out, *pos_o, *cps_o, *off_o, *sent_o, *b_o, *d_o, *unk;
  if (!PyArg_ParseTuple(args, "OO!OOOOOOO", &wt, &PyList_Type, &out, &pos_o, &cps_o, &off_o, &sent_o, &b_o, &d_o,
                        &unk))
    return NULL;
  if (check_word_type(wt) < 0) return NULL;
  Buf pos = {0}, cb = {0}, ob = {0}, sb = {0}, bb = {0}, db = {0};
  PyObject* res = NULL;
  Py_ssize_t n, ns, nc;
  if (PyObject_GetBuffer(pos_o, &pos.b, PyBUF_C_CONTIGUOUS) < 0) return NULL;
  pos.ok = 1;
  if (pos.b.itemsize != 8) {
    PyErr_SetString(PyExc_ValueError, "_ltpy.unknowns_cp: pos must be int64");
    goto done;
  }
  n = pos.b.len / 8;
  if (get_buf(cps_o, &cb, 4, 0, "cps") < 0 || get_buf(off_o, &ob, 8, 1, "off") < 0 || get_buf(sent_o, &sb, 8, n, "sent") < 0 ||
      get_buf(b_o, &bb, 8, n, "b") < 0 || get_buf(d_o, &db, 8, n, "d") < 0)
    goto done;
  ns = ob.b.len / 8 - 1;
  nc = cb.b.len / 4;
  {
    const int64_t *P = (const int64_t*)pos.b.buf, *O = (const int64_t*)ob.b.buf, *S = (const int64_t*)sb.b.buf,
                  *Bg = (const int64_t*)bb.b.buf, *D = (const int64_t*)db.b.buf;
    const uint32_t* CP = (const uint32_t*)cb.b.buf;
    const Py_ssize_t nout = PyList_GET_SIZE(out);
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (P[i] < 0 || P[i] >= nout || S[i] < 0 || S[i] >= ns || Bg[i] < 0 || D[i] < 1 ||
          O[S[i]] + Bg[i] + D[i] > O[S[i] + 1] || O[S[i] + 1] > nc) {
        PyErr_SetString(PyExc_IndexError, "_ltpy.unknowns_cp: span outside its sentence");
        goto done;
      }
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* sub = PyUnicode_FromKindAndData(PyUnicode_4BYTE_KIND, CP + O[S[i]] + Bg[i], D[i]);
      if (!sub) goto done;
      PyObject* w = new_tuple((PyTypeObject*)wt, 9);
      PyObject *ln = PyLong_FromLongLong(D[i]), *b0 = PyLong_FromLongLong(Bg[i]),
               *e0 = PyLong_FromLongLong(Bg[i] + D[i]);
      if (!w || !ln || !b0 || !e0) {
        Py_DECREF(sub);
        Py_XDECREF(w);
        Py_XDECREF(ln);
        Py_XDECREF(b0);
        Py_XDECREF(e0);
        goto done;
      }
      Py_INCREF(sub);
      PyTuple_SET_ITEM(w, 0, sub);
      PyTuple_SET_ITEM(w, 1, sub);
      Py_INCREF(Py_None);
      PyTuple_SET_ITEM(w, 2, Py_None);
      Py_INCREF(unk);
      PyTuple_SET_ITEM(w, 3, unk);
      Py_INCREF(Py_None);
      PyTuple_SET_ITEM(w, 4, Py_None);
      PyTuple_SET_ITEM(w, 5, ln);
      PyTuple_SET_ITEM(w, 6, b0);
      PyTuple_SET_ITEM(w, 7, e0);
      Py_INCREF(Py_False);
      PyTuple_SET_ITEM(w, 8, Py_False);
      untrack_atomic(w);
      PyList_SetItem(out, P[i], w);
    }
  }
  Py_INCREF(Py_None);
  res = Py_None;
done:
  rel(&pos);
  rel(&cb);
  rel(&ob);
  rel(&sb);
  rel(&bb);
  rel(&db);
  return res;
}

static PyObject* py_paths(PyObject* self, PyObject* args) {
  PyObject *flat, *ends_o, *bos, *eos, *has_o;
  if (!PyArg_ParseTuple(args, "O!OOO!O", &PyList_Type, &flat, &ends_o, &bos, &PyList_Type, &eos, &has_o))
    return NULL;
  Buf eb = {0}, hb = {0};
  PyObject* res = NULL;
  const Py_ssize_t S = PyList_GET_SIZE(eos);
  if (get_buf(ends_o, &eb, 8, S, "ends") < 0 || get_buf(has_o, &hb, 1, S, "has") < 0) goto done;
  {
    const int64_t* E = (const int64_t*)eb.b.buf;
    const uint8_t* H = (const uint8_t*)hb.b.buf;
    const Py_ssize_t nf = PyList_GET_SIZE(flat);
    int64_t a = 0;
    for (Py_ssize_t s = 0; s < S; ++s) {
      if (E[s] < a || E[s] > nf) {
        PyErr_SetString(PyExc_IndexError, "_ltpy.paths: ends not ascending within flat");
        goto done;
      }
      a = E[s];
    }
    res = PyList_New(S);
    if (!res) goto done;
    a = 0;
    PyObject** F = ((PyListObject*)flat)->ob_item;
    for (Py_ssize_t s = 0; s < S; ++s) {
      const int64_t z = E[s];
      if (!H[s]) {
        Py_INCREF(Py_None);
        PyList_SET_ITEM(res, s, Py_None);
        a = z;
        continue;
      }
      PyObject* p = PyList_New(z - a + 2);
      if (!p) {
        Py_CLEAR(res);
        goto done;
      }
      Py_INCREF(bos);
      PyList_SET_ITEM(p, 0, bos);
      for (int64_t j = a; j < z; ++j) {
        Py_INCREF(F[j]);
        PyList_SET_ITEM(p, j - a + 1, F[j]);
      }
      PyObject* e = PyList_GET_ITEM(eos, s);
      Py_INCREF(e);
      PyList_SET_ITEM(p, z - a + 1, e);
      PyList_SET_ITEM(res, s, p);
      a = z;
    }
  }
done:
  rel(&eb);
  rel(&hb);
  return res;
}

static PyObject* py_scatter(PyObject* self, PyObject* args) {
  PyObject *out, *pos_o, *vals;
  if (!PyArg_ParseTuple(args, "O!OO!", &PyList_Type, &out, &pos_o, &PyList_Type, &vals)) return NULL;
  Buf pos = {0};
  const Py_ssize_t n = PyList_GET_SIZE(vals), nout = PyList_GET_SIZE(out);
  if (get_buf(pos_o, &pos, 8, n, "pos") < 0) {
    rel(&pos);
    return NULL;
  }
  const int64_t* P = (const int64_t*)pos.b.buf;
  for (Py_ssize_t i = 0; i < n; ++i)
    if (P[i] < 0 || P[i] >= nout) {
      rel(&pos);
      PyErr_SetString(PyExc_IndexError, "_ltpy.scatter: position out of range");
      return NULL;
    }
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* v = PyList_GET_ITEM(vals, i);
    Py_INCREF(v);
    PyList_SetItem(out, P[i], v);
  }
  rel(&pos);
  Py_RETURN_NONE;
}

static PyMethodDef methods[] = {
    {"scatter", py_scatter, METH_VARARGS, "out[pos[i]] = vals[i]."},
    {"words", py_words, METH_VARARGS, "Dictionary Words into out[pos] (see module doc)."},
    {"unknowns", py_unknowns, METH_VARARGS, "Synthesised Unknown Words into out[pos]."},
    {"unknowns_cp", py_unknowns_cp, METH_VARARGS, "Unknown Words from a UTF-32 buffer into out[pos]."},
    {"paths", py_paths, METH_VARARGS, "Per-sentence path lists [bos] + flat[a:z] + [eos]."},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_ltpy", NULL, -1, methods};

PyMODINIT_FUNC PyInit__ltpy(void) { return PyModule_Create(&mod); }
