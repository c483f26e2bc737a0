// Test infrastructure: faiss::InvertedLists (FAISS 1.13.2 faiss/invlists/InvertedLists.h), the members the
// adapter uses: list_size, add_entries and the ScopedIds / ScopedCodes accessors.  See ../MetricType.h.
#pragma once
#include <cstddef>
#include <cstdint>

#include "../MetricType.h"

namespace faiss {
struct InvertedLists {
    size_t nlist;
    size_t code_size;
    InvertedLists(size_t nlist, size_t code_size);
    virtual ~InvertedLists();
    virtual size_t list_size(size_t list_no) const = 0;
    virtual const uint8_t *get_codes(size_t list_no) const = 0;
    virtual const idx_t *get_ids(size_t list_no) const = 0;
    virtual void release_codes(size_t list_no, const uint8_t *codes) const;
    virtual void release_ids(size_t list_no, const idx_t *ids) const;
    virtual size_t add_entries(size_t list_no, size_t n_entry, const idx_t *ids, const uint8_t *code) = 0;

    struct ScopedIds {
        const InvertedLists *il;
        const idx_t *ids;
        size_t list_no;
        ScopedIds(const InvertedLists *il, size_t list_no);
        const idx_t *get();
        idx_t operator[](size_t i) const;
        ~ScopedIds();
    };
    struct ScopedCodes {
        const InvertedLists *il;
        const uint8_t *codes;
        size_t list_no;
        ScopedCodes(const InvertedLists *il, size_t list_no);
        const uint8_t *get();
        ~ScopedCodes();
    };
};
}  // namespace faiss
