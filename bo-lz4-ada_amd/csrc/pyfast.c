/* _lz4ada_fast -- the streaming Update call (lz4ada_update, lz4ada.ads:281-287)
 * for Python without ctypes' per-call argument conversion: a caller that
 * feeds 4 KiB reads (tool_unlz4ada/unlz4ada.adb:16, 84-103) makes one call
 * per read, and ctypes spends ~2 us on each.  Same C-ABI underneath;
 * bo-lz4-ada_amd/lz4ada.py uses it for Decompressor.update. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include "lz4ada_hip.h"

/* update(ctx, data, start, stop, buffer) -> (status, consumed, first, last) */
static PyObject* fast_update(PyObject* self, PyObject* args)
{
	unsigned long long ctx;
	Py_buffer in, out;
	Py_ssize_t start, stop;
	(void)self;
	if (!PyArg_ParseTuple(args, "Ky*nnw*", &ctx, &in, &start, &stop, &out))
		return NULL;
	if (start < 0 || stop < start || stop > in.len) {
		PyBuffer_Release(&in);
		PyBuffer_Release(&out);
		PyErr_SetString(PyExc_ValueError, "update: 0 <= start <= stop <= len(data) required");
		return NULL;
	}
	int64_t c = 0, f = 1, l = 0;
	int st;
	const uint8_t* src = stop > start ? (const uint8_t*)in.buf + start : NULL;
	Py_BEGIN_ALLOW_THREADS
	st = lz4ada_update((lz4ada_decompressor*)(uintptr_t)ctx, src, (int64_t)(stop - start), &c,
	                   (uint8_t*)out.buf, (int64_t)out.len, &f, &l);
	Py_END_ALLOW_THREADS
	PyBuffer_Release(&in);
	PyBuffer_Release(&out);
	return Py_BuildValue("iLLL", st, (long long)c, (long long)f, (long long)l);
}

static PyMethodDef methods[] = {
	{ "update", fast_update, METH_VARARGS, "lz4ada_update over Python buffers" },
	{ NULL, NULL, 0, NULL },
};

static struct PyModuleDef module = { PyModuleDef_HEAD_INIT, "_lz4ada_fast", NULL, -1, methods };

PyMODINIT_FUNC PyInit__lz4ada_fast(void) { return PyModule_Create(&module); }
