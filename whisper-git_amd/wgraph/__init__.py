"""wgraph — MI355X commit-graph render-prep engine (host side)."""
