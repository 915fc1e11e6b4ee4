// Graph containers returned by Batch::get_graphs (reference
// common/base/include/claraparabricks/genomeworks/utils/graph.hpp:44-228).
#pragma once

#include <cstdint>
#include <map>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

namespace claraparabricks
{
namespace genomeworks
{

/// Generic labelled, weighted graph.
class Graph
{
public:
    using node_id_t     = int32_t;
    using edge_weight_t = int32_t;
    using edge_t        = std::pair<node_id_t, node_id_t>;

    const std::vector<node_id_t>& get_adjacent_nodes(node_id_t node) const
    {
        auto it = adjacent_.find(node);
        return it == adjacent_.end() ? empty_ : it->second;
    }

    const std::vector<node_id_t> get_node_ids() const
    {
        std::vector<node_id_t> ids;
        for (const auto& kv : adjacent_)
            ids.push_back(kv.first);
        return ids;
    }

    const std::vector<std::pair<edge_t, edge_weight_t>> get_edges() const
    {
        return {edges_.begin(), edges_.end()};
    }

    void set_node_label(node_id_t node, const std::string& label) { labels_.insert({node, label}); }

    std::string get_node_label(node_id_t node) const
    {
        auto it = labels_.find(node);
        return it == labels_.end() ? std::string() : it->second;
    }

protected:
    bool edge_exists(const edge_t& e) const { return edges_.count(e) != 0; }

    void link(const edge_t& e) { adjacent_[e.first].push_back(e.second); }

    void dot_body(std::ostringstream& os, const char* sep) const
    {
        for (const auto& kv : labels_)
            os << kv.first << " [label=\"" << kv.second << "\"];\n";
        for (const auto& kv : edges_)
            os << kv.first.first << " " << sep << " " << kv.first.second << " [label=\"" << kv.second << "\"];\n";
    }

    std::map<node_id_t, std::vector<node_id_t>> adjacent_;
    std::map<edge_t, edge_weight_t> edges_;
    std::map<node_id_t, std::string> labels_;
    const std::vector<node_id_t> empty_;
};

/// Directed graph (graph.hpp:186-228).
class DirectedGraph : public Graph
{
public:
    void add_edge(node_id_t from, node_id_t to, edge_weight_t weight = 0)
    {
        edge_t e(from, to);
        if (!edge_exists(e))
        {
            edges_.insert({e, weight});
            link(e);
        }
    }

    std::string serialize_to_dot() const
    {
        std::ostringstream os;
        os << "digraph g {\n";
        dot_body(os, "->");
        os << "}\n";
        return os.str();
    }
};

/// Undirected graph (graph.hpp:230-277).
class UndirectedGraph : public Graph
{
public:
    void add_edge(node_id_t a, node_id_t b, edge_weight_t weight = 0)
    {
        edge_t e(a, b), r(b, a);
        if (!edge_exists(e) && !edge_exists(r))
        {
            edges_.insert({e, weight});
            link(e);
            link(r);
        }
    }

    std::string serialize_to_dot() const
    {
        std::ostringstream os;
        os << "graph g {\n";
        dot_body(os, "--");
        os << "}\n";
        return os.str();
    }
};

} // namespace genomeworks
} // namespace claraparabricks
