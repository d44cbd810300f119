// kf.js — shared frontend runtime of the CRUD apps (the kubeflow-common-lib role, vanilla JS):
// backend calls with the CSRF double-submit header, exponential-backoff poller (1 s -> 8 s, reset
// when the data changes), namespace selection bound to the central dashboard's iframe protocol
// (library.js: parent-connected / iframe-connected / namespace-selected / all-namespaces), and the
// library's components: resource table (sortable, filterable, per-row actions, the same data-cy
// hooks as kubeflow-common-lib's resource-table), status icons (lib-status-icon semantics),
// conditions table, logs viewer, form validators (DNS-1123 names, CPU / memory quantities, limit
// >= request), snack bar, details dialog with tabs, YAML view.
//
// Every component has a pure render function (string in, string out) so node can unit-test it
// without a DOM; the DOM classes only bind those strings to elements and events.
(function (global) {
  "use strict";
  function cookie(name) {
    const m = document.cookie.match(new RegExp("(?:^|; )" + name.replace(/[-.]/g, "\\$&") + "=([^;]*)"));
    return m ? decodeURIComponent(m[1]) : "";
  }
  async function call(method, path, body) {
    const opts = { method, headers: { "Accept": "application/json" }, credentials: "same-origin" };
    if (method !== "GET") opts.headers["X-XSRF-TOKEN"] = cookie("XSRF-TOKEN");
    if (body !== undefined) {
      opts.headers["Content-Type"] = "application/json";
      opts.body = JSON.stringify(body);
    }
    const r = await fetch(path.replace(/^\//, ""), opts);
    let data = {};
    try { data = await r.json(); } catch (e) { data = { success: false, log: r.statusText }; }
    if (!r.ok || data.success === false) throw new Error(data.log || r.statusText);
    return data;
  }
  class Poller {
    constructor(fn, min = 1000, max = 8000) { this.fn = fn; this.min = min; this.max = max; this.delay = min; this.last = null; this.t = null; }
    start() { this.stop(); this.tick(); return this; }
    stop() { if (this.t) clearTimeout(this.t); this.t = null; }
    reset() { this.delay = this.min; this.start(); }
    async tick() {
      let sig = null;
      try { sig = JSON.stringify(await this.fn()); } catch (e) { console.warn(e); }
      if (sig !== null && sig !== this.last) { this.delay = this.min; this.last = sig; }
      else this.delay = Math.min(this.delay * 2, this.max);
      this.t = setTimeout(() => this.tick(), this.delay);
    }
  }
  // namespace service: inside the dashboard iframe the parent drives the selection
  const nsListeners = [];
  let currentNs = new URLSearchParams(location.search).get("ns") || localStorage.getItem("kf-namespace") || "";
  function setNamespace(ns) {
    if (!ns || ns === currentNs) return;
    currentNs = ns;
    localStorage.setItem("kf-namespace", ns);
    nsListeners.forEach((f) => f(ns));
  }
  function onNamespace(f) { nsListeners.push(f); if (currentNs) f(currentNs); }
  window.addEventListener("message", (ev) => {
    const d = ev.data || {};
    if (d.type === "namespace-selected" && d.value) setNamespace(d.value);
    if (d.type === "parent-connected" && window.parent !== window) window.parent.postMessage({ type: "iframe-connected" }, "*");
  });
  if (window.parent !== window) window.parent.postMessage({ type: "iframe-connected" }, "*");
  const icons = { ready: "&#9679;", waiting: "&#9676;", warning: "&#9888;", error: "&#10006;", stopped: "&#9632;",
                  terminating: "&#8987;", unavailable: "&#8709;", uninitialized: "&#9675;" };
  function statusCell(st) {
    st = st || {};
    return `<span class="st st-${esc(st.phase)}" title="${esc(st.message || "")}">${icons[st.phase] || "?"} ${esc(st.phase || "")}</span>`;
  }
  const esc = (v) => String(v == null ? "" : v).replace(/[&<>"']/g, (c) => ({ "&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;", "'": "&#39;" }[c]));
  // YAML view of an API object (the common-lib's Monaco YAML tab, read-only): block style, quoted
  // strings only where YAML would misread them
  function yamlScalar(v) {
    if (v === null || v === undefined) return "null";
    if (typeof v === "number" || typeof v === "boolean") return String(v);
    const s = String(v);
    if (s === "" || /^[\s\-?:,\[\]{}#&*!|>'"%@`]|[:#]\s|\s$|^(true|false|null|yes|no|on|off|~)$|^[-+]?[0-9.]+([eE][-+]?[0-9]+)?$/i.test(s) || s.includes("\n"))
      return JSON.stringify(s);
    return s;
  }
  function toYaml(v, ind = "") {
    if (Array.isArray(v)) {
      if (!v.length) return "[]";
      return v.map((x) => {
        if (x !== null && typeof x === "object" && !(Array.isArray(x) && !x.length) && Object.keys(x).length) {
          const inner = toYaml(x, ind + "  ");
          return `${ind}- ${inner.slice(ind.length + 2)}`;
        }
        return `${ind}- ${x !== null && typeof x === "object" ? (Array.isArray(x) ? "[]" : "{}") : yamlScalar(x)}`;
      }).join("\n");
    }
    if (v !== null && typeof v === "object") {
      const keys = Object.keys(v);
      if (!keys.length) return "{}";
      return keys.map((k) => {
        const x = v[k], key = yamlScalar(k);
        if (x !== null && typeof x === "object" && (Array.isArray(x) ? x.length : Object.keys(x).length))
          return `${ind}${key}:\n${toYaml(x, ind + (Array.isArray(x) ? "" : "  "))}`;
        return `${ind}${key}: ${x !== null && typeof x === "object" ? (Array.isArray(x) ? "[]" : "{}") : yamlScalar(x)}`;
      }).join("\n");
    }
    return ind + yamlScalar(v);
  }
  function eventsTable(events) {
    if (!events || !events.length) return '<p class="muted">No events.</p>';
    const rows = events.slice().sort((a, b) => String(b.lastTimestamp || "").localeCompare(String(a.lastTimestamp || "")))
      .map((e) => `<tr><td>${esc(e.type)}</td><td>${esc(e.reason)}</td><td>${esc(e.message)}</td><td>${esc(e.count || 1)}</td><td>${esc(e.lastTimestamp || e.eventTime || "")}</td></tr>`);
    return `<table class="kv"><thead><tr><th>Type</th><th>Reason</th><th>Message</th><th>Count</th><th>Last seen</th></tr></thead><tbody>${rows.join("")}</tbody></table>`;
  }
  function kvTable(pairs) {
    return `<table class="kv">${pairs.map(([k, v]) => `<tr><th>${esc(k)}</th><td>${esc(v)}</td></tr>`).join("")}</table>`;
  }
  // Resource details dialog with tabs (overview / events / logs / YAML pages of the Angular apps).
  // tabs: [{name, render: async () => html}]
  async function details(title, tabs) {
    let dlg = document.getElementById("kf-details");
    if (!dlg) {
      dlg = document.createElement("dialog");
      dlg.id = "kf-details";
      dlg.className = "details";
      document.body.append(dlg);
    }
    dlg.innerHTML = `<h2>${esc(title)}</h2><nav class="tabs">${tabs.map((t, i) => `<button data-tab="${i}">${esc(t.name)}</button>`).join("")}
      <button data-close="1" class="close">Close</button></nav><section class="tab-body"></section>`;
    const body = dlg.querySelector(".tab-body");
    async function show(i) {
      dlg.querySelectorAll("nav.tabs button[data-tab]").forEach((b) => b.classList.toggle("active", b.dataset.tab === String(i)));
      body.innerHTML = '<p class="muted">Loading…</p>';
      try { body.innerHTML = await tabs[i].render(); } catch (e) { body.innerHTML = `<p class="err">${esc(e.message)}</p>`; }
    }
    dlg.querySelectorAll("nav.tabs button[data-tab]").forEach((b) => b.addEventListener("click", () => show(Number(b.dataset.tab))));
    dlg.querySelector("button[data-close]").addEventListener("click", () => dlg.close());
    if (!dlg.open) dlg.showModal();
    await show(0);
    return dlg;
  }
  // ---- status icon (lib-status-icon: ready check_circle, stopped custom:stoppedResource,
  // unavailable timelapse, warning/error warning/error, waiting/terminating spinner) ------------
  const STATUS_ICON = { ready: "check_circle", stopped: "custom:stoppedResource", unavailable: "timelapse",
                        warning: "warning", error: "error", uninitialized: "remove_circle_outline" };
  function statusIcon(st) {
    st = st || {};
    const phase = st.phase || "";
    if (phase === "waiting" || phase === "terminating")
      return `<span class="status-icon st-${esc(phase)}" title="${esc(st.message || "")}"><span class="spinner" data-icon="spinner"></span></span>`;
    const icon = STATUS_ICON[phase] || "help";
    return `<span class="status-icon st-${esc(phase)}" title="${esc(st.message || "")}"><span class="icon" data-icon="${esc(icon)}">${icons[phase] || "?"}</span></span>`;
  }

  // ---- resource table -----------------------------------------------------------------------
  // cfg.columns: [{title, value(row) -> text (sort/filter key), html(row) -> cell html (default:
  // escaped value), sortable (default true)}]; cfg.actions: [{name, label, enabled(row)}]
  // state: {sortCol, sortDir: 1|-1, filter}. Default order: the "Name" column ascending (the
  // reference tables' default sort).
  function colValue(c, row) { return c.value ? c.value(row) : row[c.field || c.title.toLowerCase()]; }
  function sortedRows(cfg, rows, state) {
    state = state || {};
    const cols = cfg.columns;
    let idx = state.sortCol;
    if (idx === undefined || idx === null) idx = cols.findIndex((c) => c.title === "Name");
    const dir = state.sortDir || 1;
    let out = rows.slice();
    const f = (state.filter || "").trim().toLowerCase();
    if (f) out = out.filter((r) => cols.some((c) => String(colValue(c, r) == null ? "" : colValue(c, r)).toLowerCase().includes(f)));
    if (idx >= 0 && cols[idx] && cols[idx].sortable !== false) {
      const c = cols[idx];
      out.sort((a, b) => {
        const x = colValue(c, a), y = colValue(c, b);
        const nx = typeof x === "number" ? x : NaN, ny = typeof y === "number" ? y : NaN;
        const r = !isNaN(nx) && !isNaN(ny) ? nx - ny : String(x == null ? "" : x).localeCompare(String(y == null ? "" : y));
        return r * dir;
      });
    }
    return out;
  }
  function renderTable(cfg, rows, state) {
    state = state || {};
    const view = sortedRows(cfg, rows, state);
    const sortIdx = state.sortCol === undefined || state.sortCol === null ? cfg.columns.findIndex((c) => c.title === "Name") : state.sortCol;
    const head = cfg.columns.map((c, i) => {
      const arrow = i === sortIdx ? ((state.sortDir || 1) > 0 ? " &#9650;" : " &#9660;") : "";
      return `<th data-cy-table-header-row="${esc(c.title)}" data-col="${i}"${c.sortable === false ? "" : ' class="sortable"'}>${esc(c.title)}${arrow}</th>`;
    }).join("") + (cfg.actions && cfg.actions.length ? "<th></th>" : "");
    const body = view.map((r) => {
      const key = esc(cfg.key ? cfg.key(r) : (r.namespace ? r.namespace + "/" : "") + r.name);
      const cells = cfg.columns.map((c) => `<td data-cy-resource-table-row="${esc(c.title)}">${c.html ? c.html(r) : esc(colValue(c, r))}</td>`).join("");
      const acts = (cfg.actions || []).map((a) => {
        const on = a.enabled ? a.enabled(r) : true;
        return `<button data-action="${esc(a.name)}" data-key="${key}"${on ? "" : " disabled"}>${esc(typeof a.label === "function" ? a.label(r) : a.label)}</button>`;
      }).join("");
      return `<tr data-key="${key}">${cells}${cfg.actions && cfg.actions.length ? `<td class="actions">${acts}</td>` : ""}</tr>`;
    }).join("");
    const empty = view.length ? "" : `<tr><td colspan="${cfg.columns.length + 1}" class="muted">${esc(cfg.empty || "No resources.")}</td></tr>`;
    return `<table class="rt"><thead><tr>${head}</tr></thead><tbody>${body}${empty}</tbody></table>`;
  }
  // DOM binding: header click sorts (again: reverse), filter box, action buttons -> cfg.onAction
  class ResourceTable {
    constructor(el, cfg) {
      this.el = el; this.cfg = cfg; this.rows = []; this.state = { sortCol: null, sortDir: 1, filter: "" };
      el.addEventListener("click", (ev) => {
        const th = ev.target.closest("th[data-col]");
        if (th) {
          const i = Number(th.dataset.col);
          if (this.cfg.columns[i].sortable === false) return;
          const cur = this.state.sortCol === null ? this.cfg.columns.findIndex((c) => c.title === "Name") : this.state.sortCol;
          this.state.sortDir = cur === i ? -this.state.sortDir : 1;
          this.state.sortCol = i;
          this.render();
          return;
        }
        const b = ev.target.closest("button[data-action]");
        if (b && this.cfg.onAction) {
          const row = this.rows.find((r) => (this.cfg.key ? this.cfg.key(r) : (r.namespace ? r.namespace + "/" : "") + r.name) === b.dataset.key);
          if (row) this.cfg.onAction(b.dataset.action, row);
        }
        const a = ev.target.closest("a[data-open]");
        if (a && this.cfg.onOpen) {
          const row = this.rows.find((r) => (this.cfg.key ? this.cfg.key(r) : (r.namespace ? r.namespace + "/" : "") + r.name) === a.dataset.open);
          if (row) this.cfg.onOpen(row);
        }
      });
    }
    setFilter(f) { this.state.filter = f; this.render(); }
    setRows(rows) { this.rows = rows || []; this.render(); }
    render() { this.el.innerHTML = renderTable(this.cfg, this.rows, this.state); }
  }
  // the Name cell of a resource table: a link that opens the details page
  function nameLink(row) {
    return `<a class="name" data-open="${esc((row.namespace ? row.namespace + "/" : "") + row.name)}">${esc(row.name)}</a>`;
  }

  // ---- conditions table (common-lib conditions-table) -----------------------------------------
  function conditionsTable(conds) {
    if (!conds || !conds.length) return '<p class="muted">No conditions.</p>';
    const rows = conds.map((c) => {
      const ok = c.status === "True";
      return `<tr><td>${statusIcon({ phase: ok ? "ready" : "warning", message: c.status })}</td><td>${esc(c.type)}</td>` +
        `<td>${esc(c.lastTransitionTime || c.lastProbeTime || "")}</td><td>${esc(c.reason || "")}</td><td>${esc(c.message || "")}</td></tr>`;
    });
    return `<table class="kv conditions"><thead><tr><th>Status</th><th>Type</th><th>Last Transition Time</th><th>Reason</th><th>Message</th></tr></thead><tbody>${rows.join("")}</tbody></table>`;
  }

  // ---- logs viewer (common-lib logs-viewer) -----------------------------------------------------
  function renderLogs(lines, filter) {
    const f = (filter || "").toLowerCase();
    const shown = [];
    (lines || []).forEach((l, i) => { if (!f || String(l).toLowerCase().includes(f)) shown.push([i + 1, l]); });
    if (!shown.length) return '<p class="muted">No logs.</p>';
    return `<pre class="logs">${shown.map(([n, l]) => `<span class="ln">${n}</span> ${esc(l)}`).join("\n")}</pre>`;
  }
  // polls fetchLines() while following; the filter box narrows the view
  class LogsViewer {
    constructor(el, fetchLines, periodMs) { this.el = el; this.fetch = fetchLines; this.period = periodMs || 3000; this.lines = []; this.filter = ""; this.t = null; }
    async refresh() {
      try { this.lines = await this.fetch(); } catch (e) { this.el.innerHTML = `<p class="err">${esc(e.message)}</p>`; return; }
      this.el.innerHTML = renderLogs(this.lines, this.filter);
      const pre = this.el.querySelector("pre");
      if (pre) pre.scrollTop = pre.scrollHeight;
    }
    follow() { this.stop(); const tick = async () => { await this.refresh(); this.t = setTimeout(tick, this.period); }; tick(); return this; }
    stop() { if (this.t) clearTimeout(this.t); this.t = null; }
  }

  // ---- form validators (common-lib form/validators) -------------------------------------------
  const DNS1123 = /^[a-z0-9]([-a-z0-9]*[a-z0-9])?$/;
  const QTY = /^([0-9]+(\.[0-9]+)?|\.[0-9]+)(m|k|M|G|T|P|E|Ki|Mi|Gi|Ti|Pi|Ei)?$/;
  const SUFFIX = { m: 1e-3, k: 1e3, M: 1e6, G: 1e9, T: 1e12, P: 1e15, E: 1e18,
                   Ki: 1024, Mi: 1024 ** 2, Gi: 1024 ** 3, Ti: 1024 ** 4, Pi: 1024 ** 5, Ei: 1024 ** 6 };
  function parseQuantity(q) {
    const s = String(q == null ? "" : q).trim();
    const m = s.match(QTY);
    if (!m) return NaN;
    return parseFloat(m[1]) * (m[3] ? SUFFIX[m[3]] : 1);
  }
  const validators = {
    name(v, maxLen) {
      const s = String(v || "");
      if (!s) return "Name is required";
      if (s.length > (maxLen || 63)) return `Name must be at most ${maxLen || 63} characters`;
      if (!DNS1123.test(s)) return "Name must consist of lowercase alphanumeric characters or '-', and must start and end with an alphanumeric character";
      return "";
    },
    cpu(v) { return isNaN(parseQuantity(v)) || parseQuantity(v) <= 0 ? `Invalid CPU value: ${v}` : ""; },
    memory(v) { return isNaN(parseQuantity(v)) || parseQuantity(v) <= 0 ? `Invalid memory value: ${v}` : ""; },
    limitAtLeastRequest(request, limit, what) {
      if (limit === "" || limit == null) return "";
      return parseQuantity(limit) < parseQuantity(request) ? `${what} limit must be greater than or equal to the request` : "";
    },
  };

  // ---- snack bar ------------------------------------------------------------------------------
  function snack(message, status) {
    let el = document.getElementById("kf-snack");
    if (!el) { el = document.createElement("div"); el.id = "kf-snack"; document.body.append(el); }
    el.className = "snack";
    el.setAttribute("data-cy-snack-status", status || "INFO");
    el.textContent = message;
    el.hidden = false;
    clearTimeout(el._t);
    el._t = setTimeout(() => { el.hidden = true; }, status === "ERROR" ? 8000 : 3000);
  }

  function h(tag, attrs, ...children) {
    const e = document.createElement(tag);
    Object.entries(attrs || {}).forEach(([k, v]) => (k.startsWith("on") ? e.addEventListener(k.slice(2), v) : e.setAttribute(k, v)));
    children.flat().forEach((c) => e.append(c instanceof Node ? c : document.createTextNode(String(c))));
    return e;
  }
  global.kf = { call, Poller, cookie, setNamespace, onNamespace, namespace: () => currentNs, statusCell, h,
                esc, toYaml, eventsTable, kvTable, details, statusIcon, renderTable, sortedRows, ResourceTable, nameLink,
                conditionsTable, renderLogs, LogsViewer, validators, parseQuantity, snack };
  if (typeof module !== "undefined" && module.exports) module.exports = global.kf;  // node unit tests
})(typeof window !== "undefined" ? window : globalThis);
