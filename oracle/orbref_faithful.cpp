/*
 * orbref_faithful.cpp -- TEST INFRASTRUCTURE ONLY (parity oracle; never linked into liborbx).
 *
 * ORBextractor::DistributeOctTree (src/ORBextractor.cc:644-907) with the reference's own data
 * structures: ExtractorNode objects in a std::list, children pushed to the front, and the
 * "split the largest nodes first" phase sorting std::pair<int, ExtractorNode*> (:815).  That sort
 * breaks ties between equal-size nodes by the nodes' heap addresses, so the kept keypoints (and
 * their order) depend on where malloc put the list nodes.
 *
 * orbref.c's orbref_distribute breaks those ties by creation order instead (the canonical order
 * the GPU kernel K3 reproduces).  This file exists to MEASURE how often the two disagree under a
 * real allocator (glibc malloc here, as in the reference's process): tests/test_quadtree_ties.py.
 *
 * The node layout mirrors include/ORBextractor.h:32-43 (a 28-byte keypoint like cv::KeyPoint, four
 * 8-byte points, a list iterator, a bool), so the list nodes and key vectors take the same malloc
 * size classes as the reference's.  The keypoint's class_id slot carries the candidate index.
 */
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <list>
#include <utility>
#include <vector>

namespace {

struct Key {   // cv::KeyPoint: Point2f pt; float size, angle, response; int octave, class_id
    float x, y, size, angle, response;
    int octave, class_id;
};
static_assert(sizeof(Key) == 28, "cv::KeyPoint layout");

struct Pt {
    int x, y;
};

struct Node {
    Node() : bNoMore(false), seq(0) {}
    void divide(Node& n1, Node& n2, Node& n3, Node& n4) const;
    std::vector<Key> vKeys;
    Pt UL, UR, BL, BR;
    std::list<Node>::iterator lit;
    bool bNoMore;
    int seq;   // creation order (tie_mode 1 only); fits the padding after bNoMore, so sizeof(Node) is unchanged
};
static_assert(sizeof(Node) == 72, "ExtractorNode layout (vector, 4 points, iterator, bool)");

int g_seq = 0;

// ExtractorNode::DivideNode, src/ORBextractor.cc:569-629
void Node::divide(Node& n1, Node& n2, Node& n3, Node& n4) const
{
    const int halfX = (int)std::ceil(static_cast<float>(UR.x - UL.x) / 2);
    const int halfY = (int)std::ceil(static_cast<float>(BR.y - UL.y) / 2);
    n1.UL = UL;
    n1.UR = Pt{UL.x + halfX, UL.y};
    n1.BL = Pt{UL.x, UL.y + halfY};
    n1.BR = Pt{UL.x + halfX, UL.y + halfY};
    n1.vKeys.reserve(vKeys.size());
    n2.UL = n1.UR;
    n2.UR = UR;
    n2.BL = n1.BR;
    n2.BR = Pt{UR.x, UL.y + halfY};
    n2.vKeys.reserve(vKeys.size());
    n3.UL = n1.BL;
    n3.UR = n1.BR;
    n3.BL = BL;
    n3.BR = Pt{n1.BR.x, BL.y};
    n3.vKeys.reserve(vKeys.size());
    n4.UL = n3.UR;
    n4.UR = n2.BR;
    n4.BL = n3.BR;
    n4.BR = BR;
    n4.vKeys.reserve(vKeys.size());
    for (const Key& kp : vKeys) {
        if (kp.x < n1.UR.x) {
            if (kp.y < n1.BR.y) n1.vKeys.push_back(kp);
            else n3.vKeys.push_back(kp);
        } else if (kp.y < n1.BR.y) {
            n2.vKeys.push_back(kp);
        } else {
            n4.vKeys.push_back(kp);
        }
    }
    if (n1.vKeys.size() == 1) n1.bNoMore = true;
    if (n2.vKeys.size() == 1) n2.bNoMore = true;
    if (n3.vKeys.size() == 1) n3.bNoMore = true;
    if (n4.vKeys.size() == 1) n4.bNoMore = true;
}

typedef std::vector<std::pair<int, Node*> > SizePtr;

// push the non-empty children to the front of the list (n1..n4 order); nodes with more than one
// key are recorded for the next round.  Returns how many were recorded.
int link(std::list<Node>& l, Node* ch, SizePtr& rec)
{
    int n = 0;
    for (int q = 0; q < 4; ++q) {
        if (ch[q].vKeys.empty()) continue;
        ch[q].seq = g_seq++;
        l.push_front(ch[q]);
        if (ch[q].vKeys.size() > 1) {
            ++n;
            rec.push_back(std::make_pair((int)ch[q].vKeys.size(), &l.front()));
            l.front().lit = l.begin();
        }
    }
    return n;
}

}  // namespace

// tie_mode 0: the reference's (size, heap address) sort; 1: (size, creation order), which must reproduce
// orbref_distribute exactly (the check that this restatement differs from it only in the tie-break).
extern "C" int orbref_distribute_faithful(const int* xys, int n, int minX, int maxX, int minY, int maxY, int N,
                                          int tie_mode, int* out, int cap)
{
    g_seq = 0;
    // :650-653
    const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
    if (nIni <= 0) return -1;
    const float hX = static_cast<float>(maxX - minX) / nIni;

    std::list<Node> lNodes;
    std::vector<Node*> vpIniNodes(nIni);
    for (int i = 0; i < nIni; i++) {   // :663-675
        Node ni;
        ni.UL = Pt{(int)(hX * static_cast<float>(i)), 0};
        ni.UR = Pt{(int)(hX * static_cast<float>(i + 1)), 0};
        ni.BL = Pt{ni.UL.x, maxY - minY};
        ni.BR = Pt{ni.UR.x, maxY - minY};
        ni.vKeys.reserve(n);
        ni.seq = g_seq++;
        lNodes.push_back(ni);
        vpIniNodes[i] = &lNodes.back();
    }
    for (int k = 0; k < n; k++) {   // :679-683
        const Key kp{(float)xys[3 * k], (float)xys[3 * k + 1], 7.f, -1.f, (float)xys[3 * k + 2], 0, k};
        size_t r = (size_t)(kp.x / hX);
        if (r >= (size_t)nIni) r = (size_t)nIni - 1;
        vpIniNodes[r]->vKeys.push_back(kp);
    }
    for (std::list<Node>::iterator lit = lNodes.begin(); lit != lNodes.end();) {   // :688-699
        if (lit->vKeys.size() == 1) {
            lit->bNoMore = true;
            ++lit;
        } else if (lit->vKeys.empty()) {
            lit = lNodes.erase(lit);
        } else {
            ++lit;
        }
    }

    bool bFinish = false;
    SizePtr vSizeAndPointerToNode;
    vSizeAndPointerToNode.reserve(lNodes.size() * 4);
    while (!bFinish) {   // :710-876
        int prevSize = (int)lNodes.size();
        int nToExpand = 0;
        vSizeAndPointerToNode.clear();
        for (std::list<Node>::iterator lit = lNodes.begin(); lit != lNodes.end();) {
            if (lit->bNoMore) {
                ++lit;
                continue;
            }
            Node ch[4];
            lit->divide(ch[0], ch[1], ch[2], ch[3]);
            nToExpand += link(lNodes, ch, vSizeAndPointerToNode);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if (((int)lNodes.size() + nToExpand * 3) > N) {
            while (!bFinish) {   // :805-874
                prevSize = (int)lNodes.size();
                SizePtr vPrev = vSizeAndPointerToNode;
                vSizeAndPointerToNode.clear();
                if (tie_mode == 0)
                    std::sort(vPrev.begin(), vPrev.end());   // (size, heap address)
                else
                    std::sort(vPrev.begin(), vPrev.end(), [](const std::pair<int, Node*>& a, const std::pair<int, Node*>& b) {
                        return a.first != b.first ? a.first < b.first : a.second->seq < b.second->seq;
                    });
                for (int j = (int)vPrev.size() - 1; j >= 0; j--) {
                    Node ch[4];
                    vPrev[j].second->divide(ch[0], ch[1], ch[2], ch[3]);
                    link(lNodes, ch, vSizeAndPointerToNode);
                    lNodes.erase(vPrev[j].second->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }

    // :882-906 the best keypoint per node (first maximum wins), in list order
    int m = 0;
    for (const Node& nd : lNodes) {
        const Key* best = &nd.vKeys[0];
        float maxResponse = best->response;
        for (size_t k = 1; k < nd.vKeys.size(); k++)
            if (nd.vKeys[k].response > maxResponse) {
                best = &nd.vKeys[k];
                maxResponse = nd.vKeys[k].response;
            }
        if (m >= cap) return -1;
        out[m++] = best->class_id;
    }
    return m;
}
