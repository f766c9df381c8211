// dataflow.h -- the simulation harness's linear element chain (host only, no GPU knowledge).
// The CLI (main.cpp) and the harness elements (viterbiDF.h) are written against the reference's
// src/dataflow/dataflow.h interface, so this keeps its names and printed report: ComputeElement with
// process() / probe() / a per-element status map, Pipeline built with operator|, run() returning the
// final output plus the outputs of probed elements, printStatus() with each element's "Elapsed run time".
#pragma once

#include <any>
#include <chrono>
#include <cstdio>
#include <functional>
#include <iostream>
#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <typeinfo>
#include <vector>

using OptData = std::optional<std::any>;

namespace dataflow_detail {
// "12.34 s" / "56.78 ms" / "910 us", as the reference's report prints an element's run time
inline std::string elapsed_text(std::chrono::microseconds d)
{
    const long long us = d.count();
    char buf[64];
    if (us > 1000000) std::snprintf(buf, sizeof buf, "%.2f s", us * 1e-6);
    else if (us > 1000) std::snprintf(buf, sizeof buf, "%.2f ms", us * 1e-3);
    else std::snprintf(buf, sizeof buf, "%lld us", us);
    return buf;
}
constexpr const char* kElapsed = "Elapsed run time";
}  // namespace dataflow_detail

// One element of the chain: a source when its input is empty (std::nullopt), else a transform.
class ComputeElement {
    std::map<std::string, std::any> entries_;
    bool tapped_ = false;

public:
    virtual ~ComputeElement() = default;
    virtual std::any process(const OptData& in) = 0;

    // mark the element so that Pipeline::run keeps a copy of its output
    ComputeElement& probe()
    {
        tapped_ = true;
        return *this;
    }
    bool isProbed() const { return tapped_; }

    void setStatus(const std::string& key, std::any v) { entries_[key] = std::move(v); }
    std::any getStatus(const std::string& key) const { return entries_.at(key); }
    const std::map<std::string, std::any>& getStatusMap() const { return entries_; }

    // elements override this for the status entries they know how to print
    virtual std::string getStatusString(const std::string&) const { return "(Not printable)"; }
    std::string getStatusStringAll(const std::string& key) const
    {
        if (key == dataflow_detail::kElapsed)
            return dataflow_detail::elapsed_text(std::any_cast<std::chrono::microseconds>(entries_.at(key)));
        return getStatusString(key);
    }
};

struct PipelineResult {
    std::any final_output;
    std::vector<std::any> probed_outputs;
};

class Pipeline {
    std::vector<std::reference_wrapper<ComputeElement>> chain_;

public:
    Pipeline& add(ComputeElement& e)
    {
        chain_.emplace_back(e);
        return *this;
    }

    // each element's output feeds the next; every element's wall time goes into its status map
    PipelineResult run()
    {
        PipelineResult out;
        OptData data;
        for (ComputeElement& e : chain_) {
            const auto begin = std::chrono::high_resolution_clock::now();
            data = e.process(data);
            e.setStatus(dataflow_detail::kElapsed, std::chrono::duration_cast<std::chrono::microseconds>(
                                                       std::chrono::high_resolution_clock::now() - begin));
            if (e.isProbed()) out.probed_outputs.push_back(*data);
        }
        if (!data.has_value()) throw std::runtime_error("Pipeline produced no output");
        out.final_output = std::move(*data);
        return out;
    }

    void printStatus() const
    {
        std::cout << "--- Pipeline Status ---\n";
        size_t idx = 0;
        for (const ComputeElement& e : chain_) {
            std::cout << "Element " << idx++ << " (type: " << typeid(e).name() << "):\n";
            if (e.getStatusMap().empty()) std::cout << "  - No status information.\n";
            for (const auto& entry : e.getStatusMap())
                std::cout << "  - " << entry.first << ": " << e.getStatusStringAll(entry.first) << "\n";
        }
        std::cout << "--- End of Status ---\n";
    }
};

inline Pipeline operator|(ComputeElement& first, ComputeElement& second)
{
    Pipeline p;
    p.add(first).add(second);
    return p;
}
inline Pipeline operator|(Pipeline p, ComputeElement& next)
{
    p.add(next);
    return p;
}
