// Match.hpp -- drop-in for the reference's P/Match.hpp:1-14.
//
// Same class name, member names, member order and constructor signature, so
// brace-init call sites like Matcher.push_back({ i, j, v }) (P/Main.cpp:418)
// compile unchanged; layout {unsigned, unsigned, double} = 16 bytes, identical
// to usv_match in usv.h (checked against the reference's own compiled
// P/Match.cpp in tests/test_match_layout.py).
#ifndef Match_HPP
#define Match_HPP

class Match {
public:
    Match(unsigned int LeftIndex, unsigned int RightIndex, double MatchValue);
    unsigned int LeftIndex;
    unsigned int RightIndex;
    double MatchValue;
};

#endif /* Match_HPP */
