"""ORACLE package -- test infrastructure only (see deequ_oracle.py / oracle.c headers)."""
