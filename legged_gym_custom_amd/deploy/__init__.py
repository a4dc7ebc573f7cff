"""Single-robot deployment side: the reference's deploy/base package
(config_parser.py, deploy_base.py) — the numpy observation builder a real or MuJoCo
controller runs, with the scan-replay ("fake scan") state machine. Reachable under the
reference's module path `deploy.base.*` through the root `deploy` alias package."""
