"""The reference's known-answer tables (tests/golden/reference_kats.json, written by
tests/golden/make_golden.py) and the names of the tables that are raft.tryCommit calls."""
import json
import os

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))

# every table of commit_case records (one raft.tryCommit call each)
COMMIT_TABLES = [
    "TestCommit", "TestLeaderOnlyCommitsLogFromCurrentTerm", "TestLeaderAcknowledgeCommit",
    "TestLeaderCommitPrecedingEntries", "TestSingleNodeCommit",
    "TestCannotCommitWithoutNewTermEntry", "TestCommitWithoutNewTermEntry", "TestLeaderAppResp",
    "TestFullMemberWithOneWitness", "TestVotingMemberLengthMismatch", "TestCommitAfterRemoveNode",
    "TestCommitTo", "TestTryCommitResetsMatchArray",
]


def commit_cases():
    return [c for t in COMMIT_TABLES for c in KATS[t]]
