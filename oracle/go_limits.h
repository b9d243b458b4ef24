/* ORACLE — test infrastructure only.  Go regexp/syntax parse-size limits
 * (ErrLarge, ErrNestingDepth) replayed on Go's parse shapes; go_limits.c. */
#ifndef BJX_GO_LIMITS_H
#define BJX_GO_LIMITS_H
#include <stdint.h>

typedef struct GoLim GoLim;
GoLim *golim_new(int (*fold)(int));
void golim_free(GoLim *g);
/* 0 = within the limits, 1 = ErrLarge, 2 = ErrNestingDepth (sticky) */
int golim_failed(const GoLim *g);
/* parser events; flags = Go's FoldCase (1) | NonGreedy (32) | WasDollar (256) */
void golim_literal(GoLim *g, int c, unsigned flags);
void golim_op(GoLim *g, int op, unsigned flags, int cap);
void golim_class(GoLim *g, const int *pairs, int n_pairs, unsigned flags);
void golim_esc_alloc(GoLim *g);
void golim_esc_class(GoLim *g, const int *pairs, int n_pairs, unsigned flags);
void golim_esc_free(GoLim *g);
void golim_vertical_bar(GoLim *g, unsigned flags);
void golim_right_paren(GoLim *g, unsigned flags);
void golim_repeat(GoLim *g, int op, int min, int max, unsigned flags);
void golim_end(GoLim *g, unsigned flags);
#endif
