// Deterministic synthetic matrices for the benchmark configurations
// (BASELINE.json configs C3-C5; generator spec in DESIGN.md §5).
//
// splitmix64_at(seed, i) is the i-th (0-based) output of the splitmix64
// generator started at state `seed`; every element is a pure function of its
// global position, so row-partitioned shards generate exactly the rows of the
// whole matrix.
#ifndef SPMV_AMD_SYNTHETIC_H_
#define SPMV_AMD_SYNTHETIC_H_

#include <cstdint>
#include <vector>

uint64_t splitmix64_at(uint64_t seed, uint64_t i);
// U[-1, 1): (z >> 11) * 2^-52 - 1, exact in f64.
double uniform11(uint64_t z);

// "Stripe" uniform random CSR: global row r has k distinct sorted columns, one
// per stripe [j*cols/k, (j+1)*cols/k): col_j = lo_j + splitmix64_at(seedCol,
// r*k+j) mod (hi_j - lo_j); value uniform11(splitmix64_at(seedVal, r*k+j)).
// Fills rows [row0, row0+nrows) with rowptr rebased to 0.
void genStripeCSR(uint64_t row0, uint32_t nrows, uint32_t cols, uint32_t k, uint64_t seedCol, uint64_t seedVal,
                  uint32_t* rowptr, uint32_t* colind, double* vals);

// Graph500-style R-MAT, 2^scale x 2^scale, edgeFactor * 2^scale edges drawn
// with quadrant probabilities (a, b, c, d); duplicates summed (in edge order),
// columns ascending within rows, values uniform11.  Returns nnz.
uint64_t genRmatCSR(uint32_t scale, uint32_t edgeFactor, uint64_t seed, double a, double b, double c,
                    std::vector<uint32_t>& rowptr, std::vector<uint32_t>& colind, std::vector<double>& vals);

// The same matrix restricted to rows [row0, row1) (rowptr rebased to 0,
// columns global): what a rank of a row-partitioned run generates.  Every
// edge is still drawn (the row of an edge is only known once drawn), in
// parallel; equal to the corresponding rows of genRmatCSR.
uint64_t genRmatCSRRows(uint32_t scale, uint32_t edgeFactor, uint64_t seed, double a, double b, double c,
                        uint32_t row0, uint32_t row1, std::vector<uint32_t>& rowptr, std::vector<uint32_t>& colind,
                        std::vector<double>& vals);

// Edges per row before duplicates are summed (counts[2^scale]): the input of
// an nnz-balanced partition that no rank has to materialise the matrix for.
void genRmatRowCounts(uint32_t scale, uint32_t edgeFactor, uint64_t seed, double a, double b, double c,
                      uint32_t* counts);

// nnz-balanced contiguous row partition: bounds[0..parts], bounds[0] = 0,
// bounds[parts] = rows, each part holding about nnz/parts nonzeros; interior
// bounds are multiples of HIPSPMV_SHARD_ALIGN (64) rows, the nearer one.
void partitionRows(const uint32_t* rowptr, uint32_t rows, uint32_t parts, uint32_t* bounds);
// Same from per-row counts: bounds[p] = first row whose prefix count reaches
// total*p/parts, snapped the same way.
void partitionRowCounts(const uint32_t* counts, uint32_t rows, uint32_t parts, uint32_t* bounds);

// Worker threads of the host generators: $SPMV_THREADS, else
// $OMP_NUM_THREADS, else min(16, hardware threads).
unsigned hostThreads();

#endif
