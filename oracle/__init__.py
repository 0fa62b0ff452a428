"""ORACLE — test infrastructure only (CPU restatements of the reference used
as the parity checker and as bench.py's cpu_baseline).  The product package
`dqn_mgsc_zoo_amd` never imports anything from here."""
