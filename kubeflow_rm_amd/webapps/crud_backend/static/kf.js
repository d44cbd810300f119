// kf.js — shared frontend runtime of the CRUD apps (the kubeflow-common-lib role, vanilla JS):
// backend calls with the CSRF double-submit header, exponential-backoff poller (1 s -> 8 s, reset
// when the data changes), namespace selection bound to the central dashboard's iframe protocol
// (library.js: parent-connected / iframe-connected / namespace-selected / all-namespaces), status
// icons and small DOM helpers.
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
  function h(tag, attrs, ...children) {
    const e = document.createElement(tag);
    Object.entries(attrs || {}).forEach(([k, v]) => (k.startsWith("on") ? e.addEventListener(k.slice(2), v) : e.setAttribute(k, v)));
    children.flat().forEach((c) => e.append(c instanceof Node ? c : document.createTextNode(String(c))));
    return e;
  }
  global.kf = { call, Poller, cookie, setNamespace, onNamespace, namespace: () => currentNs, statusCell, h,
                esc, toYaml, eventsTable, kvTable, details };
  if (typeof module !== "undefined" && module.exports) module.exports = global.kf;  // node unit tests
})(typeof window !== "undefined" ? window : globalThis);
