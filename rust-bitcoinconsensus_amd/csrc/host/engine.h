// Internal interface of the batch engine (engine.cpp), shared with the workload builder.
#pragma once
#include <cstddef>
#include <vector>

#include "../pipeline.h"
#include "bitcoinconsensus.h"

namespace bcc {
namespace host {

// Deserializes and checks the items (flags / deserialize / index / size, in reference order) and
// runs the interpreter once with the deferring checker.  jobs / rows receive every deferred ECDSA
// check (the first GPU round of bitcoinconsensus_verify_batch); tuple_item[k] = item of row k.
// Returns the number of deferred tuples.
size_t build_first_round(const bcc_batch_item* items, size_t n, unsigned flags, SighashJobs& jobs,
                         TupleRows& rows, std::vector<uint32_t>* tuple_item = nullptr);

// Appends src (jobs + rows) to dst, fixing offsets / indices.
void append_round(SighashJobs& dst, TupleRows& dst_rows, const SighashJobs& src,
                  const TupleRows& src_rows);

// Frees the calling thread's Taproot job buffers (host/taproot.cpp).
void taproot_release_thread_state();

}  // namespace host
}  // namespace bcc
