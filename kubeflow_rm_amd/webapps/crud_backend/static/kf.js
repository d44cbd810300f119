// kf.js — shared frontend runtime of the CRUD apps (the kubeflow-common-lib role, vanilla JS):
// backend calls with the CSRF double-submit header, exponential-backoff poller (1 s -> 8 s, reset
// when the data changes), namespace selection bound to the central dashboard's iframe protocol
// (library.js: parent-connected / iframe-connected / namespace-selected / all-namespaces), and the
// library's components: resource table (sortable; chip filter: every term must match, "text"
// against any column, "column:value" against one; paginated 10 / 20 / 50; per-row actions; the
// same data-cy hooks as kubeflow-common-lib's resource-table; date-time and memory cells),
// status icons (lib-status-icon semantics), conditions table, logs viewer, form validators
// (DNS-1123 names, CPU / memory quantities, limit >= request), confirm dialog with its applying /
// error states, snack bar, details dialog with tabs, YAML view.
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
    if (s === "" || /^[\s\-?:,\[\]{}#&*!|>'"%@`]|[:#]\s|\s#|\s$|^(true|false|null|yes|no|on|off|~)$|^[-+]?[0-9.]+([eE][-+]?[0-9]+)?$/i.test(s) || s.includes("\n"))
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
  // ---- YAML editor (lib-monaco-editor, language "yaml") and loader (js-yaml load as used by the
  // apps' shared/utils/yaml.ts parseYAML) ---------------------------------------------------------
  // parseYaml covers the block YAML the apps exchange: mappings, sequences (also compact "- k: v"
  // items and sequences at their key's indent), plain scalars with the core-schema types, quoted
  // scalars, one-line flow collections, | and > block scalars, comments and "---". It returns
  // [value, ""] or [{}, "<reason> (line:column)"]; empty text is [{}, ""] (the reference contract).
  function yamlError(msg, line, col) { return new Error(`${msg} (${line + 1}:${(col || 0) + 1})`); }
  function stripComment(s) {
    let q = null;
    for (let i = 0; i < s.length; i++) {
      const c = s[i];
      if (q) {
        if (q === '"' && c === "\\") i++;
        else if (q === "'" && c === "'" && s[i + 1] === "'") i++;
        else if (c === q) q = null;
      } else if ((c === '"' || c === "'") && (i === 0 || /[\s[{,:]/.test(s[i - 1]))) q = c;
      else if (c === "#" && (i === 0 || /\s/.test(s[i - 1]))) return s.slice(0, i).replace(/\s+$/, "");
    }
    return s.replace(/\s+$/, "");
  }
  function plainScalar(s) {
    if (s === "" || s === "~" || /^(null|Null|NULL)$/.test(s)) return null;
    if (/^(true|True|TRUE)$/.test(s)) return true;
    if (/^(false|False|FALSE)$/.test(s)) return false;
    if (/^[-+]?[0-9]+$/.test(s)) return parseInt(s, 10);
    if (/^0x[0-9a-fA-F]+$/.test(s)) return parseInt(s.slice(2), 16);
    if (/^0o[0-7]+$/.test(s)) return parseInt(s.slice(2), 8);
    if (/^[-+]?(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?$/.test(s)) return parseFloat(s);
    if (/^[-+]?\.(inf|Inf|INF)$/.test(s)) return s[0] === "-" ? -Infinity : Infinity;
    if (/^\.(nan|NaN|NAN)$/.test(s)) return NaN;
    return s;
  }
  // a quoted scalar that must span all of s
  function quotedScalar(s, line, col) {
    if (s[0] === '"') {
      const m = s.match(/^"((?:[^"\\]|\\.)*)"$/);
      if (m) { try { return JSON.parse(`"${m[1].replace(/\\'/g, "'")}"`); } catch (e) { /* below */ } }
      throw yamlError("bad double-quoted scalar", line, col);
    }
    const m = s.match(/^'((?:[^']|'')*)'$/);
    if (!m) throw yamlError("bad single-quoted scalar", line, col);
    return m[1].replace(/''/g, "'");
  }
  // one-line flow collection: [a, "b", {c: 1}]
  function flowValue(s, line, col) {
    let i = 0;
    const ws = () => { while (i < s.length && /\s/.test(s[i])) i++; };
    const fail = (what) => yamlError(what, line, col + i);
    function token(isKey) {
      ws();
      if (s[i] === '"' || s[i] === "'") {
        const q = s[i];
        let j = i + 1;
        for (; j < s.length; j++) {
          if (q === '"' && s[j] === "\\") j++;
          else if (q === "'" && s[j] === "'" && s[j + 1] === "'") j++;
          else if (s[j] === q) break;
        }
        if (j >= s.length) throw fail("unterminated quoted scalar");
        const t = s.slice(i, j + 1);
        i = j + 1;
        return quotedScalar(t, line, col);
      }
      let j = i;
      while (j < s.length && !/[,\]}]/.test(s[j]) && !(isKey && s[j] === ":")) j++;
      const t = s.slice(i, j).trim();
      i = j;
      return isKey ? t : plainScalar(t);
    }
    function value() {
      ws();
      if (s[i] === "[" || s[i] === "{") {
        const seq = s[i] === "[", close = seq ? "]" : "}", out = seq ? [] : {};
        i++;
        for (;;) {
          ws();
          if (s[i] === close) { i++; return out; }
          if (seq) out.push(value());
          else {
            const k = token(true);
            ws();
            let v = null;
            if (s[i] === ":") { i++; v = value(); }
            out[k] = v;
          }
          ws();
          if (s[i] === ",") { i++; continue; }
          if (s[i] === close) { i++; return out; }
          throw fail(`missed comma between flow collection entries`);
        }
      }
      return token(false);
    }
    const v = value();
    ws();
    if (i < s.length) throw fail("unexpected characters after a flow collection");
    return v;
  }
  function loadYaml(text) {
    const raw = String(text).replace(/\r\n?/g, "\n").split("\n");
    const L = [];
    raw.forEach((r, n) => {
      const lead = r.match(/^[ \t]*/)[0];
      const t = stripComment(r);
      if (!t.trim() || /^(---|\.\.\.)(\s|$)/.test(t)) return;
      if (lead.includes("\t")) throw yamlError("tab characters must not be used in indentation", n, lead.indexOf("\t"));
      L.push({ n, ind: lead.length, t: t.trim() });
    });
    if (!L.length) return null;
    let i = 0;
    const isSeq = (t) => t === "-" || t.startsWith("- ");
    const isHeader = (t) => /^[|>][-+]?[0-9]?$/.test(t);
    // "key: rest" -> [key, rest] (rest "" for a nested node), null when t is no mapping entry
    function splitKey(t, ln) {
      let k, j;
      if (t[0] === '"' || t[0] === "'") {
        const q = t[0];
        for (j = 1; j < t.length; j++) {
          if (q === '"' && t[j] === "\\") j++;
          else if (q === "'" && t[j] === "'" && t[j + 1] === "'") j++;
          else if (t[j] === q) break;
        }
        const rest = t.slice(j + 1).match(/^\s*:(\s+|$)/);
        if (!rest) return null;
        k = quotedScalar(t.slice(0, j + 1), ln.n, ln.ind);
        return [k, t.slice(j + 1 + rest[0].length).trim()];
      }
      if (/^[[{]/.test(t) || isSeq(t)) return null;
      const m = t.match(/^(.*?):(\s+|$)/);
      if (!m) return null;
      return [m[1].trim(), t.slice(m[0].length).trim()];
    }
    function scalar(t, ln, col) {
      if (t[0] === '"' || t[0] === "'") return quotedScalar(t, ln.n, col);
      if (t[0] === "[" || t[0] === "{") return flowValue(t, ln.n, col);
      return plainScalar(t);
    }
    // | and > content: the raw lines after ln deeper than the parent's indent
    function blockScalar(header, parentInd, ln) {
      const lines = [];
      let last = ln.n, contentInd = -1;
      for (let n = ln.n + 1; n < raw.length; n++) {
        const r = raw[n];
        if (!r.trim()) { lines.push(""); continue; }
        const ind = r.match(/^ */)[0].length;
        if (ind <= parentInd) break;
        if (contentInd < 0) contentInd = ind;
        if (ind < contentInd) throw yamlError("bad indentation of a block scalar line", n, ind);
        lines.push(r.slice(contentInd));
        last = n;
      }
      lines.length = Math.max(0, last - ln.n);  // trailing blank lines belong to chomping, not content
      while (i < L.length && L[i].n <= last) i++;
      let body;
      if (header[0] === "|") body = lines.join("\n");
      else {
        body = "";
        lines.forEach((l, k) => {
          if (k === 0) body = l;
          else if (l === "") body += "\n";
          else body += (body.endsWith("\n") || body === "" ? "" : " ") + l;
        });
      }
      const chomp = header.includes("-") ? "" : "\n";
      return body === "" ? "" : body + chomp;
    }
    function node(minInd) {
      const ln = L[i];
      if (ln.ind < minInd) return null;
      if (isSeq(ln.t)) return seq(ln.ind);
      if (splitKey(ln.t, ln)) return map(ln.ind);
      i++;
      return scalar(ln.t, ln, ln.ind);
    }
    function child(ind, ln) {  // the nested node of an entry with no inline value
      if (i < L.length && L[i].ind > ind) return node(L[i].ind);
      return null;
    }
    function seq(ind) {
      const out = [];
      while (i < L.length && L[i].ind === ind && isSeq(L[i].t)) {
        const ln = L[i];
        const rest = ln.t === "-" ? "" : ln.t.slice(1).trimStart();
        const col = ind + ln.t.length - rest.length;
        if (!rest) { i++; out.push(child(ind, ln)); }
        else if (isSeq(rest) || splitKey(rest, ln)) { L[i] = { n: ln.n, ind: col, t: rest }; out.push(node(col)); }
        else if (isHeader(rest)) { i++; out.push(blockScalar(rest, ind, ln)); }
        else { i++; out.push(scalar(rest, ln, col)); }
      }
      if (i < L.length && L[i].ind > ind) throw yamlError("bad indentation of a sequence entry", L[i].n, L[i].ind);
      return out;
    }
    function map(ind) {
      const out = {};
      while (i < L.length && L[i].ind === ind) {
        const ln = L[i];
        const kv = splitKey(ln.t, ln);
        if (!kv) throw yamlError(isSeq(ln.t) ? "bad indentation of a sequence entry" : "can not read a block mapping entry", ln.n, ln.ind);
        const [k, rest] = kv;
        if (Object.prototype.hasOwnProperty.call(out, k)) throw yamlError("duplicated mapping key", ln.n, ln.ind);
        i++;
        if (!rest) out[k] = i < L.length && L[i].ind === ind && isSeq(L[i].t) ? seq(ind) : child(ind, ln);
        else if (isHeader(rest)) out[k] = blockScalar(rest, ind, ln);
        else out[k] = scalar(rest, ln, ind + ln.t.length - rest.length);
      }
      if (i < L.length && L[i].ind > ind) throw yamlError("bad indentation of a mapping entry", L[i].n, L[i].ind);
      return out;
    }
    const v = node(0);
    if (i < L.length) throw yamlError("end of the stream or a document separator is expected", L[i].n, L[i].ind);
    return v;
  }
  function parseYaml(text) {
    if (!text) return [{}, ""];
    try { return [loadYaml(text), ""]; } catch (e) { return [{}, e.message]; }
  }
  // token-coloured HTML of YAML text (keys, strings, numbers / booleans / null, comments, dashes)
  function highlightYaml(text) {
    return String(text).split("\n").map((line) => {
      const body = stripComment(line), comment = line.slice(body.length);
      const m = body.match(/^(\s*(?:- +)*)(.*)$/);
      let out = esc(m[1]).replace(/-/g, '<span class="y-p">-</span>');
      let rest = m[2];
      const kv = rest.match(/^((?:"(?:[^"\\]|\\.)*"|'(?:[^']|'')*'|[^\s"'[{#][^:]*?))(\s*:)(\s+|$)(.*)$/);
      if (kv) { out += `<span class="y-k">${esc(kv[1])}</span>${esc(kv[2] + kv[3])}`; rest = kv[4]; }
      const v = rest.trim();
      if (v) {
        const cls = /^["']/.test(v) ? "y-s" : /^[[{|>]/.test(v) ? "y-f"
          : (typeof plainScalar(v) !== "string" ? "y-n" : "y-v");
        out += `<span class="${cls}">${esc(rest)}</span>`;
      }
      return out + (comment.trim() ? `${esc(comment.slice(0, comment.indexOf("#")))}<span class="y-c">${esc(comment.slice(comment.indexOf("#")))}</span>` : esc(comment));
    }).join("\n");
  }
  // static read-only editor markup (gutter + highlight) for tabs that need no interaction
  function yamlHtml(text, height) {
    const t = String(text == null ? "" : text);
    const gutter = Array.from({ length: t.split("\n").length }, (_, k) => k + 1).join("\n");
    return `<div class="yaml-editor ro" style="height:${Number(height) || 490}px"><pre class="gutter">${gutter}</pre>` +
      `<div class="code"><pre class="hl">${highlightYaml(t)}\n</pre></div></div>`;
  }
  // Editor over a host element: line-number gutter + highlighted text; editable (a textarea laid
  // over the highlight) unless readOnly. onChange(text, value, error) on every edit; the parse
  // error shows under the editor (the apps' mat-error "errorParsingYaml").
  class YamlEditor {
    constructor(el, opts) {
      this.el = el;
      this.opts = opts || {};
      const ro = !!this.opts.readOnly;
      el.innerHTML = `<div class="yaml-editor${ro ? " ro" : ""}" style="height:${Number(this.opts.height) || 250}px">` +
        `<pre class="gutter"></pre><div class="code"><pre class="hl"></pre>${ro ? "" : '<textarea spellcheck="false" wrap="off"></textarea>'}</div></div>` +
        '<p class="yaml-error err" data-cy="yaml-error"></p>';
      this.ta = el.querySelector("textarea");
      if (this.ta) {
        this.ta.addEventListener("input", () => this.setText(this.ta.value, true));
        this.ta.addEventListener("keydown", (ev) => {  // Tab indents by two spaces instead of leaving the field
          if (ev.key !== "Tab" || typeof this.ta.selectionStart !== "number") return;
          ev.preventDefault();
          const a = this.ta.selectionStart, b = this.ta.selectionEnd, v = this.ta.value;
          this.ta.value = v.slice(0, a) + "  " + v.slice(b);
          this.ta.selectionStart = this.ta.selectionEnd = a + 2;
          this.setText(this.ta.value, true);
        });
      }
      this.setText(this.opts.text || "", false);
    }
    setText(text, fromUser) {
      this.text = String(text == null ? "" : text);
      [this.value, this.error] = parseYaml(this.text);
      const n = this.text.split("\n").length;
      this.el.querySelector(".gutter").textContent = Array.from({ length: n }, (_, k) => k + 1).join("\n");
      this.el.querySelector(".hl").innerHTML = highlightYaml(this.text) + "\n";
      this.el.querySelector(".yaml-error").textContent = this.error;
      if (this.ta && this.ta.value !== this.text) this.ta.value = this.text;
      if (fromUser && this.opts.onChange) this.opts.onChange(this.text, this.value, this.error);
    }
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
  // column kinds: "date" (lib DateTimeValue: "5 minutes ago", full time on hover, sorted by time)
  // and "memory" (MemoryValue: a quantity shown in binary units, sorted by bytes)
  function colValue(c, row) { return c.value ? c.value(row) : row[c.field || c.title.toLowerCase()]; }
  function sortKey(c, row) {
    const v = colValue(c, row);
    if (c.kind === "date") { const t = Date.parse(v); return isNaN(t) ? -Infinity : t; }
    if (c.kind === "memory") { try { return quantityToScalar(v); } catch (e) { return NaN; } }
    return v;
  }
  function viewText(c, row) {
    const v = colValue(c, row);
    if (c.kind === "memory") { try { return formatBytes(quantityToScalar(v)); } catch (e) { return String(v); } }
    return v == null ? "" : String(v);
  }
  // the filter box holds comma-separated chips: "ready" matches any column, "status:ready" only
  // the Status column (table.component.ts filterPredicate: all chips AND-ed)
  function parseFilter(text) {
    return String(text || "").split(",").map((t) => t.trim().toLowerCase()).filter(Boolean).map((t) => {
      const i = t.indexOf(":");
      return i > 0 && i < t.length - 1 ? { column: t.slice(0, i), value: t.slice(i + 1) } : t;
    });
  }
  function cellMatches(c, row, needle) {
    if (viewText(c, row).toLowerCase().includes(needle)) return true;
    return c.kind === "date" && !!colValue(c, row) && timeAgo(colValue(c, row)).toLowerCase().includes(needle);
  }
  function rowMatches(cols, row, terms) {
    return terms.every((t) => (typeof t === "string"
      ? cols.some((c) => cellMatches(c, row, t))
      : cols.some((c) => c.title.toLowerCase() === t.column && cellMatches(c, row, t.value))));
  }
  function sortedRows(cfg, rows, state) {
    state = state || {};
    const cols = cfg.columns;
    let idx = state.sortCol;
    if (idx === undefined || idx === null) idx = cols.findIndex((c) => c.title === "Name");
    const dir = state.sortDir || 1;
    let out = rows.slice();
    const terms = parseFilter(state.filter);
    if (terms.length) out = out.filter((r) => rowMatches(cols, r, terms));
    if (idx >= 0 && cols[idx] && cols[idx].sortable !== false) {
      const c = cols[idx];
      out.sort((a, b) => {
        const x = sortKey(c, a), y = sortKey(c, b);
        const nx = typeof x === "number" ? x : NaN, ny = typeof y === "number" ? y : NaN;
        const r = !isNaN(nx) && !isNaN(ny) ? nx - ny : String(x == null ? "" : x).localeCompare(String(y == null ? "" : y));
        return r * dir;
      });
    }
    return out;
  }
  // mat-paginator: page sizes 10 / 20 / 50 (default 50), "1 – 10 of 23"
  const PAGE_SIZES = [10, 20, 50];
  function paginate(total, page, size) {
    size = PAGE_SIZES.includes(size) ? size : 50;
    const pages = Math.max(1, Math.ceil(total / size));
    page = Math.min(Math.max(0, page || 0), pages - 1);
    const start = page * size, end = Math.min(total, start + size);
    return { page, size, pages, start, end, label: total ? `${start + 1} – ${end} of ${total}` : "0 of 0" };
  }
  function renderCell(c, r) {
    if (c.html) return c.html(r);
    if (c.kind === "date") return dateTimeHtml(colValue(c, r));
    return esc(viewText(c, r));
  }
  function renderTable(cfg, rows, state) {
    state = state || {};
    const all = sortedRows(cfg, rows, state);
    const pg = paginate(all.length, state.page, state.pageSize);
    const view = all.slice(pg.start, pg.end);
    const sortIdx = state.sortCol === undefined || state.sortCol === null ? cfg.columns.findIndex((c) => c.title === "Name") : state.sortCol;
    const head = cfg.columns.map((c, i) => {
      const arrow = i === sortIdx ? ((state.sortDir || 1) > 0 ? " &#9650;" : " &#9660;") : "";
      return `<th data-cy-table-header-row="${esc(c.title)}" data-col="${i}"${c.sortable === false ? "" : ' class="sortable"'}>${esc(c.title)}${arrow}</th>`;
    }).join("") + (cfg.actions && cfg.actions.length ? "<th></th>" : "");
    const body = view.map((r) => {
      const key = esc(cfg.key ? cfg.key(r) : (r.namespace ? r.namespace + "/" : "") + r.name);
      const cells = cfg.columns.map((c) => `<td data-cy-resource-table-row="${esc(c.title)}">${renderCell(c, r)}</td>`).join("");
      const acts = (cfg.actions || []).map((a) => {
        const on = a.enabled ? a.enabled(r) : true;
        return `<button data-action="${esc(a.name)}" data-key="${key}"${on ? "" : " disabled"}>${esc(typeof a.label === "function" ? a.label(r) : a.label)}</button>`;
      }).join("");
      return `<tr data-key="${key}">${cells}${cfg.actions && cfg.actions.length ? `<td class="actions">${acts}</td>` : ""}</tr>`;
    }).join("");
    const empty = view.length ? "" : `<tr><td colspan="${cfg.columns.length + 1}" class="muted">${esc(cfg.empty || "No resources.")}</td></tr>`;
    const pager = all.length > PAGE_SIZES[0] ? `<div class="paginator" data-cy-paginator>` +
      `<label>Items per page <select data-page-size>${PAGE_SIZES.map((n) => `<option${n === pg.size ? " selected" : ""}>${n}</option>`).join("")}</select></label>` +
      `<span class="range">${pg.label}</span>` +
      `<button data-page="prev"${pg.page > 0 ? "" : " disabled"}>&lsaquo;</button><button data-page="next"${pg.page < pg.pages - 1 ? "" : " disabled"}>&rsaquo;</button></div>` : "";
    return `<table class="rt"><thead><tr>${head}</tr></thead><tbody>${body}${empty}</tbody></table>${pager}`;
  }
  // DOM binding: header click sorts (again: reverse), filter box, action buttons -> cfg.onAction
  class ResourceTable {
    constructor(el, cfg) {
      this.el = el; this.cfg = cfg; this.rows = []; this.state = { sortCol: null, sortDir: 1, filter: "", page: 0, pageSize: 50 };
      el.addEventListener("change", (ev) => {
        if (ev.target.matches && ev.target.matches("select[data-page-size]")) {
          this.state.pageSize = Number(ev.target.value);
          this.state.page = 0;
          this.render();
        }
      });
      el.addEventListener("click", (ev) => {
        const pb = ev.target.closest("button[data-page]");
        if (pb) {
          this.state.page += pb.dataset.page === "next" ? 1 : -1;
          this.render();
          return;
        }
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
    setFilter(f) { this.state.filter = f; this.state.page = 0; this.render(); }
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

  // ---- quantities and bytes (resource-table MemoryValue) ----------------------------------------
  // Kubernetes quantity -> number ("500m" -> 0.5, "1Gi" -> 1073741824); unknown suffix throws
  const QTY_SCALE = { n: 1e-9, u: 1e-6, m: 1e-3, "": 1, k: 1e3, M: 1e6, G: 1e9, T: 1e12, P: 1e15, E: 1e18,
                      Ki: 2 ** 10, Mi: 2 ** 20, Gi: 2 ** 30, Ti: 2 ** 40, Pi: 2 ** 50, Ei: 2 ** 60 };
  function quantityToScalar(q) {
    if (q === undefined || q === null || q === "") return 0;
    const m = String(q).trim().match(/^([+-]?(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?)([a-zA-Z]*)$/);
    if (!m || !(m[2] in QTY_SCALE)) throw new Error(`Unknown quantity ${q}`);
    return Number(m[1]) * QTY_SCALE[m[2]];
  }
  // bytes -> "1.5 Gi" (binary units, one decimal) or "1.6 GB" with si
  function formatBytes(bytes, si, decimals) {
    const base = si ? 1000 : 1024, d = decimals === undefined ? 1 : decimals;
    if (Math.abs(bytes) < base) return `${bytes} B`;
    const units = si ? ["kB", "MB", "GB", "TB", "PB", "EB"] : ["Ki", "Mi", "Gi", "Ti", "Pi", "Ei"];
    let u = -1, v = bytes;
    const r = 10 ** d;
    do { v /= base; u++; } while (Math.round(Math.abs(v) * r) / r >= base && u < units.length - 1);
    return `${v.toFixed(d)} ${units[u]}`;
  }

  // ---- date-time (lib-date-time: distance in words with a suffix, "about" / "almost" dropped) --
  function timeAgo(date, now) {
    const t = date instanceof Date ? date.getTime() : Date.parse(date);
    if (!date || isNaN(t)) return "-";
    const ref = now === undefined ? Date.now() : typeof now === "number" ? now : now instanceof Date ? now.getTime() : Date.parse(now);
    const secs = Math.abs(ref - t) / 1000, mins = Math.round(secs / 60);
    const plural = (n, w) => `${n} ${w}${n === 1 ? "" : "s"}`;
    let words;
    if (mins < 1) words = "less than a minute";
    else if (mins < 45) words = plural(mins, "minute");
    else if (mins < 90) words = "1 hour";
    else if (mins < 1440) words = plural(Math.round(mins / 60), "hour");
    else if (mins < 2520) words = "1 day";
    else if (mins < 43200) words = plural(Math.round(mins / 1440), "day");
    else if (mins < 86400) words = plural(Math.round(mins / 43200), "month");
    else {
      const a = new Date(Math.min(t, ref)), b = new Date(Math.max(t, ref));
      let months = (b.getUTCFullYear() - a.getUTCFullYear()) * 12 + b.getUTCMonth() - a.getUTCMonth();
      if (b.getUTCDate() < a.getUTCDate()) months -= 1;
      if (months < 12) words = plural(Math.round(mins / 43200), "month");
      else {
        const years = Math.floor(months / 12), rest = months % 12;
        words = rest < 3 ? plural(years, "year") : rest < 9 ? `over ${plural(years, "year")}` : plural(years + 1, "year");
      }
    }
    return ref >= t ? `${words} ago` : `in ${words}`;
  }
  // a date cell: relative time, the local and UTC time on hover (the component's popover)
  function dateTimeHtml(date) {
    if (!date) return "-";
    const t = Date.parse(date);
    const local = isNaN(t) ? String(date) : new Date(t).toString();
    return `<span class="date-time" data-date="${esc(date)}" title="Local: ${esc(local)}&#10;UTC: ${esc(date)}">${esc(timeAgo(date))}</span>`;
  }

  // ---- confirm dialog (lib-confirm-dialog) -------------------------------------------------------
  // cfg: {title, message, accept, cancel, applying, confirmColor, error}. The accept button turns
  // into a disabled "applying" button while onAccept runs; a failure keeps the dialog open with
  // the error under the message (the apps' delete / stop / close-viewer flows).
  function renderConfirm(cfg, applying) {
    return `<h2 class="dialog-title">${esc(cfg.title)}</h2><div class="dialog-content"><p>${esc(cfg.message || "")}</p>` +
      `<p class="error" data-cy-dialog-error>${esc(cfg.error || "")}</p></div><div class="dialog-actions">` +
      `<button data-resp="cancel">${esc(String(cfg.cancel || "cancel").toUpperCase())}</button>` +
      (applying
        ? `<button disabled class="applying"><span class="spinner"></span> ${esc(String(cfg.applying || "").toUpperCase())}</button>`
        : `<button data-resp="accept" class="${esc(cfg.confirmColor || "primary")}">${esc(String(cfg.accept || "ok").toUpperCase())}</button>`) +
      "</div>";
  }
  function confirmDialog(cfg, onAccept) {
    return new Promise((resolve) => {
      const dlg = document.createElement("dialog");
      dlg.className = "confirm";
      if (cfg.width) dlg.style.width = cfg.width;
      document.body.append(dlg);
      const state = Object.assign({}, cfg);
      const done = (resp) => { dlg.close(); dlg.remove(); resolve(resp); };
      const draw = (applying) => {
        dlg.innerHTML = renderConfirm(state, applying);
        const cancel = dlg.querySelector('button[data-resp="cancel"]');
        cancel.onclick = () => done("cancel");
        const ok = dlg.querySelector('button[data-resp="accept"]');
        if (ok) ok.onclick = async () => {
          draw(true);
          try { if (onAccept) await onAccept(); done("accept"); }
          catch (e) { state.error = e.message || String(e); draw(false); }
        };
      };
      dlg.addEventListener("cancel", () => done("cancel"));
      draw(false);
      dlg.showModal();
    });
  }

  // an information dialog: heading (+ sub-heading), arbitrary content, one CLOSE button
  function infoDialog(heading, subHeading, html, width) {
    const dlg = document.createElement("dialog");
    dlg.className = "info";
    if (width) dlg.style.width = width;
    document.body.append(dlg);
    dlg.innerHTML = `<h2 class="dialog-title">${esc(heading)} <span class="muted">${esc(subHeading || "")}</span></h2>` +
      `<div class="dialog-content">${html}</div><div class="dialog-actions"><button data-resp="close">CLOSE</button></div>`;
    const done = () => { dlg.close(); dlg.remove(); };
    dlg.querySelector('button[data-resp="close"]').onclick = done;
    dlg.addEventListener("cancel", done);
    dlg.showModal();
    return dlg;
  }

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
                conditionsTable, renderLogs, LogsViewer, validators, parseQuantity, snack, parseFilter, rowMatches,
                paginate, PAGE_SIZES, quantityToScalar, formatBytes, timeAgo, dateTimeHtml, renderConfirm, confirmDialog, infoDialog,
                parseYaml, highlightYaml, yamlHtml, YamlEditor };
  if (typeof module !== "undefined" && module.exports) module.exports = global.kf;  // node unit tests
})(typeof window !== "undefined" ? window : globalThis);
