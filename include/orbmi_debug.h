/*
 * orbmi debug hooks — stage-level views used by the parity tests (tests/) to localise a
 * mismatch inside ORBextractor::operator().  Not part of the reference interface.
 */
#ifndef ORBMI_DEBUG_H
#define ORBMI_DEBUG_H
#include "orbmi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* FAST candidates of `level` of batch item `item` of the last extraction, before
 * DistributeOctTree, in the reference's vToDistributeKeys order (src/ORBextractor.cc:778-829):
 * xyr = {x, y, score} int triples with x, y relative to minBorder (16, 16). */
int orbmi_debug_fast_candidates(orbmi_extractor* h, int item, int level, int* xyr, int cap, int* n_out);

/* Keypoints kept by DistributeOctTree for `level` (level coordinates, list order):
 * xyr = {x, y, score} triples. */
int orbmi_debug_octree_level(orbmi_extractor* h, int item, int level, int* xyr, int cap, int* n_out);

#ifdef __cplusplus
}
#endif
#endif
