#include "SpMV.h"

// software/SpMV.cpp:3-12: the base class only records the operands.
SpMV::SpMV(SparseMatrix* A, SpMVData* x, SpMVData* y) : m_A(A), m_x(x), m_y(y) {}

SpMV::~SpMV() {}
