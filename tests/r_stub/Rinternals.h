/* Declarations of the R C API subset used by src/ccg_r.c -- for a
 * syntax/type check of the glue only (R is not installed in this image). */
#pragma once
#include <stddef.h>
#include <stdio.h>
typedef struct SEXPREC* SEXP;
typedef ptrdiff_t R_xlen_t;
typedef unsigned int SEXPTYPE;
#define INTSXP 13
#define REALSXP 14
#define STRSXP 16
#define VECSXP 19
#define EXTPTRSXP 22
#define TRUE 1
#define FALSE 0
typedef int Rboolean;
extern int R_NaInt;
#define NA_INTEGER R_NaInt
extern double R_NaReal;
#define NA_REAL R_NaReal
extern SEXP R_NilValue;
extern SEXP R_NamesSymbol;
SEXP Rf_install(const char*);
SEXP Rf_allocVector(SEXPTYPE, R_xlen_t);
SEXP Rf_allocMatrix(SEXPTYPE, int, int);
SEXP Rf_ScalarInteger(int);
SEXP Rf_ScalarReal(double);
SEXP Rf_mkChar(const char*);
SEXP Rf_protect(SEXP);
void Rf_unprotect(int);
#define PROTECT(s) Rf_protect(s)
#define UNPROTECT(n) Rf_unprotect(n)
int* INTEGER(SEXP);
double* REAL(SEXP);
int TYPEOF(SEXP);
R_xlen_t XLENGTH(SEXP);
int Rf_length(SEXP);
int Rf_nrows(SEXP);
int Rf_ncols(SEXP);
int Rf_asInteger(SEXP);
double Rf_asReal(SEXP);
int Rf_asLogical(SEXP);
SEXP VECTOR_ELT(SEXP, R_xlen_t);
SEXP SET_VECTOR_ELT(SEXP, R_xlen_t, SEXP);
void SET_STRING_ELT(SEXP, R_xlen_t, SEXP);
SEXP Rf_setAttrib(SEXP, SEXP, SEXP);
void* R_ExternalPtrAddr(SEXP);
SEXP R_ExternalPtrTag(SEXP);
SEXP R_MakeExternalPtr(void*, SEXP, SEXP);
void R_ClearExternalPtr(SEXP);
typedef void (*R_CFinalizer_t)(SEXP);
void R_RegisterCFinalizerEx(SEXP, R_CFinalizer_t, Rboolean);
void __attribute__((noreturn)) Rf_error(const char*, ...);
char* R_alloc(size_t, int);
