/* ORACLE — test infrastructure only. Go regexp restatement (see go_regexp.c). */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gre gre;

/* regexp.Compile (syntax.Perl flags). NULL + Go-style message on error. */
gre *gre_compile(const char *pat, size_t len, char *err, size_t errlen);
int gre_parse_check(const char *pat, size_t len, char *err, size_t errlen);
/* (*Regexp).Match on a byte slice: 1 if any match, else 0. */
int gre_match(const gre *g, const uint8_t *text, size_t len);
void gre_free(gre *g);

#ifdef __cplusplus
}
#endif
