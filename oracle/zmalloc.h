/* Forced include for the zero-initialised reference build (SURVEY.md §0 finding 1, §8 c1).
 * The reference never initialises Symbol.deleted (histogram.cpp:14-22 of the reference) nor
 * several Trainer fields, so a stock build's merge order depends on heap garbage.  Making every
 * malloc a calloc is the only source-free way to give the reference well-defined behaviour. */
#include <stdlib.h>
#define malloc(n) calloc(1, (n))
