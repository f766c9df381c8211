// dataflow.h -- minimal linear element pipeline for the simulation harness.
// Interface-compatible with the reference's src/dataflow/dataflow.h (ComputeElement, Pipeline,
// PipelineResult, operator|, probe(), per-element status with "Elapsed run time"), so the CLI and
// viterbiDF.h read the same; host-only, no GPU knowledge.
#pragma once

#include <any>
#include <chrono>
#include <iomanip>
#include <iostream>
#include <map>
#include <optional>
#include <sstream>
#include <stdexcept>
#include <string>
#include <typeinfo>
#include <vector>

using OptData = std::optional<std::any>;

class ComputeElement {
public:
    virtual ~ComputeElement() = default;
    // in == std::nullopt for a source element
    virtual std::any process(const OptData& in) = 0;

    ComputeElement& probe() { probed_ = true; return *this; }
    bool isProbed() const { return probed_; }

    void setStatus(const std::string& key, std::any v) { status_[key] = std::move(v); }
    std::any getStatus(const std::string& key) const { return status_.at(key); }
    const std::map<std::string, std::any>& getStatusMap() const { return status_; }

    virtual std::string getStatusString(const std::string&) const { return "(Not printable)"; }
    std::string getStatusStringAll(const std::string& key) const
    {
        if (key != "Elapsed run time") return getStatusString(key);
        const double us = (double)std::any_cast<std::chrono::microseconds>(status_.at(key)).count();
        std::ostringstream os;
        os << std::fixed << std::setprecision(2);
        if (us > 1e6) os << us / 1e6 << " s";
        else if (us > 1e3) os << us / 1e3 << " ms";
        else os << std::setprecision(0) << us << " us";
        return os.str();
    }

protected:
    std::map<std::string, std::any> status_;

private:
    bool probed_ = false;
};

struct PipelineResult {
    std::any final_output;
    std::vector<std::any> probed_outputs;
};

class Pipeline {
public:
    Pipeline& add(ComputeElement& e) { stages_.push_back(&e); return *this; }

    PipelineResult run()
    {
        PipelineResult r;
        OptData cur;
        for (ComputeElement* e : stages_) {
            const auto t0 = std::chrono::high_resolution_clock::now();
            cur = e->process(cur);
            const auto t1 = std::chrono::high_resolution_clock::now();
            e->setStatus("Elapsed run time", std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0));
            if (e->isProbed()) r.probed_outputs.push_back(*cur);
        }
        if (!cur) throw std::runtime_error("Pipeline produced no output");
        r.final_output = std::move(*cur);
        return r;
    }

    void printStatus() const
    {
        std::cout << "--- Pipeline Status ---\n";
        for (size_t i = 0; i < stages_.size(); i++) {
            std::cout << "Element " << i << " (type: " << typeid(*stages_[i]).name() << "):\n";
            const auto& m = stages_[i]->getStatusMap();
            if (m.empty()) std::cout << "  - No status information.\n";
            for (const auto& kv : m) std::cout << "  - " << kv.first << ": " << stages_[i]->getStatusStringAll(kv.first) << "\n";
        }
        std::cout << "--- End of Status ---\n";
    }

private:
    std::vector<ComputeElement*> stages_;
};

inline Pipeline operator|(ComputeElement& a, ComputeElement& b) { Pipeline p; p.add(a).add(b); return p; }
inline Pipeline operator|(Pipeline p, ComputeElement& b) { p.add(b); return p; }
