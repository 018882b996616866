/* ref_quiet.c -- TEST INFRASTRUCTURE ONLY (the "quiet" reference baseline).
 *
 * The reference prints debug lines on its hot path (math_util.c rkf45_integrate: ~20 per
 * attempt; raytracer.c: per ray). Linked into _ref/libref.so with -Bsymbolic, these no-op
 * definitions take those calls (gcc may emit printf as puts/putchar, or __printf_chk under
 * _FORTIFY_SOURCE), so the CPU baseline times the arithmetic, not stdio formatting. The
 * library is loaded RTLD_LOCAL (ctypes), so nothing else in the process binds to them. */
#include <stdarg.h>
#include <stdio.h>

int printf(const char* fmt, ...) {
    (void)fmt;
    return 0;
}

int puts(const char* s) {
    (void)s;
    return 0;
}

int putchar(int c) {
    return c;
}

int __printf_chk(int flag, const char* fmt, ...) {
    (void)flag;
    (void)fmt;
    return 0;
}
