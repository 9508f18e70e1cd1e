/* Host-only sanitizer run of the oracle (test infrastructure, not product
 * code): oracle/sst_oracle.c compiled with -fsanitize=address,undefined into
 * this driver, which calls every entry point the tests use on a canonical +
 * modification alphabet (is_valid, explain with and without the memo,
 * recursion, both length bounds) and prints a checksum.  Built and run by
 * tests/test_oracle_asan.py. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct ora_result {
  int status;
  int64_t n_solutions, n_empty, n_items, lookups;
  int32_t* lens;
  int16_t* rows;
} ora_result;

int64_t ora_table_cols(int64_t max_mass, int C);
int ora_build_table(const int64_t* masses, int n, int64_t max_mass, int C, void* out);
int ora_is_valid(const void* table, int nrows, int64_t cols, int C, double mass, double threshold, double tolerance,
                 double precision);
void ora_result_free(ora_result* r);
int ora_explain_table(const void* table, int nrows, int64_t cols, int C, const int64_t* w, const uint8_t* is_mod,
                      const int64_t* cap, double mass, double threshold, double tolerance, double precision, int64_t A,
                      int with_memo, int store, ora_result* out);
int ora_explain_recursion(int nrows, const int64_t* w, const uint8_t* is_mod, const int64_t* cap, double mass,
                          double threshold, double tolerance, double precision, int64_t A, ora_result* out);
int64_t ora_length_bound(const void* table, int nrows, int64_t cols, int C, const int64_t* w, const uint8_t* is_mod,
                         const int64_t* cap, double su_mass, double obs_mass, double tolerance, double precision,
                         int64_t max_len, int64_t max_mods, int dir);

int main(void) {
  const int64_t w[] = {0, 305042, 306026, 320045, 329053, 345048, 359062, 384093};
  const uint8_t mod[] = {0, 0, 0, 1, 0, 0, 1, 1};
  const int64_t cap[] = {0, 10, 10, 3, 10, 10, 2, 1};
  const int n = 8, C = 32;
  const int64_t max_mass = 384093 * 35, cols = ora_table_cols(max_mass, C);
  void* table = calloc((size_t)n * (size_t)cols, C / 4);
  if (!table || ora_build_table(w, n, max_mass, C, table) != 0) return 2;
  uint64_t sum = 0;
  srand(7);
  for (int i = 0; i < 300; ++i) {
    const int k = 1 + rand() % 6;
    double m = 0.0;
    for (int j = 0; j < k; ++j) m += (double)w[1 + rand() % (n - 1)] * 1e-3;
    m += ((rand() % 2001) - 1000) * 1e-6;
    const double thr = 1e-5 * (1000.0 + rand() % 8000);
    sum += (uint64_t)(ora_is_valid(table, n, cols, C, m, thr, 1e-5, 1e-3) + 2);
    for (int memo = 0; memo < 2; ++memo) {
      ora_result r;
      ora_explain_table(table, n, cols, C, w, mod, cap, m, thr, 1e-5, 1e-3, (i % 4) ? 3 : -1, memo, 1, &r);
      sum = sum * 31 + (uint64_t)r.n_solutions + 7 * (uint64_t)r.n_items;
      ora_result_free(&r);
    }
    if (i % 15 == 0) {
      ora_result r;
      ora_explain_recursion(n, w, mod, cap, m, thr, 1e-5, 1e-3, 3, &r);
      sum = sum * 31 + (uint64_t)r.n_solutions;
      ora_result_free(&r);
    }
    if (i % 30 == 0)
      for (int dir = 0; dir < 2; ++dir)
        sum = sum * 31 + (uint64_t)(ora_length_bound(table, n, cols, C, w, mod, cap, m, m, 1e-5, 1e-3, 12, 4, dir) + 9);
  }
  free(table);
  printf("checksum %llu\n", (unsigned long long)sum);
  return 0;
}
